"""A/B of library builds on one box: lockstep ms/step of the config-2
workload, each build in its own process (HTM_AMD_LIB_VARIANT), interleaved
over rounds (cdna_hip_programming.md §5.4 rule 24: same box, alternating).
usage: python tools/ab_libs.py <variant|main>[@ENV=VAL...] ...   (main = libhtm_amd.so)
The engine reads ENV=VAL knobs only in builds with -DHTM_AB_KNOBS: "ab@HTM_FLUSH_WG=64"
(make -C <pkg>/csrc ab -> libhtm_amd_ab.so); "main@..." is refused."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time, json
import numpy as np, torch
sys.path.insert(0, ROOT)
import _pkg, bench
rt = _pkg.load()
N, K = int(os.environ.get("AB_STREAMS", "1024")), int(os.environ.get("AB_STEPS", "128"))
R = int(os.environ.get("AB_REGIONS", "3"))
d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
train = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))][:2184]
trace = d["test_cpu"].astype(np.float64)
eng, _, _, _ = bench.trained_engine(rt, N, 72 * 1024, 0, train)
eng.set_learning(False, False)
vals = torch.tensor(bench.make_inputs(N, 0, N, 0, 16 + R * K, trace), device="cuda")
for k in range(16):
    eng.step(vals[k])
torch.cuda.synchronize()
ts = []
for r in range(R):
    t0 = time.perf_counter()
    out = [eng.step(vals[16 + r * K + k]) for k in range(K)]
    eng.flush()
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) / K * 1e3)
h = float(torch.stack(out).double().sum().item())
print(json.dumps({"ms": ts, "checksum": h}))
'''.replace("ROOT", repr(ROOT))
variants = sys.argv[1:] or ["main", "prev"]
rounds = int(os.environ.get("AB_ROUNDS", "3"))
res = {v: [] for v in variants}
sums = {}
for r in range(rounds):
    for v in variants:
        env = dict(os.environ)
        env.pop("HTM_AMD_LIB_VARIANT", None)
        lib, *kv = v.split("@")  # "<build>@ENV=VAL@..." sets engine env knobs too
        if kv and lib == "main":
            sys.exit("env knobs need the A/B build: use ab@... (make ab)")
        if lib != "main":
            env["HTM_AMD_LIB_VARIANT"] = lib
        for x in kv:
            k_, v_ = x.split("=", 1)
            env[k_] = v_
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=400)
        if p.returncode != 0:
            print(p.stderr[-2000:], file=sys.stderr)
            sys.exit(p.returncode)
        o = json.loads(p.stdout.strip().splitlines()[-1])
        res[v] += o["ms"]
        sums[v] = o["checksum"]
        print(v, [round(x, 4) for x in o["ms"]], flush=True)
print(json.dumps({"median_ms": {v: round(float(np.median(x)), 4) for v, x in res.items()},
                  "ms": {v: [round(a, 4) for a in x] for v, x in res.items()},
                  "checksums_equal": len(set(sums.values())) == 1}))
