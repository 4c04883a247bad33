# per-phase stamps of the default (push) and non-returning (np) qualification builds
set -o pipefail
T=${AB_TAG:-st}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u tools/stamps.py > gpurun_out/$T/stamps_push.json 2>gpurun_out/$T/stamps_push.err || exit 1
HTM_AMD_LIB=libhtm_amd_stnp.so timeout -k 10 300 python -u tools/stamps.py > gpurun_out/$T/stamps_np.json 2>/dev/null || exit 1
