"""First-contact GPU diagnostic: step the HIP engine and the oracle side by
side on the Model-1 training trace and report the first divergence."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import _pkg  # noqa: E402
import oracle  # noqa: E402

rt = _pkg.load()
N_TRAIN = int(os.environ.get("DIAG_TRAIN", "300"))
N_TEST = int(os.environ.get("DIAG_TEST", "100"))


def cmp_state(eng, orc, tag):
    bad = []
    a = eng.tm_states(0)
    b = orc.tm_states()
    for k in a:
        if not np.array_equal(a[k], b[k]):
            bad.append(f"{k}: gpu {a[k].sum()} orc {b[k].sum()} diff {np.nonzero(a[k] != b[k])[0][:8]}")
    ca, cb = eng.col_confidence(0), orc.col_confidence()
    if not np.array_equal(ca, cb):
        d = np.nonzero(ca != cb)[0]
        bad.append(f"colconf differs at {len(d)} cols e.g. {d[:5]} {ca[d[:3]]} vs {cb[d[:3]]}")
    sa, sb = eng.tm_segments(0), orc.tm_segments(32)
    if len(sa["cell"]) != len(sb["cell"]):
        bad.append(f"nseg gpu {len(sa['cell'])} orc {len(sb['cell'])}")
    else:
        for k in ["cell", "is_seq", "pos_act", "last_dc_iter", "nsyn", "last_dc", "src", "perm"]:
            if not np.array_equal(sa[k], sb[k]):
                idx = np.nonzero((sa[k] != sb[k]).reshape(len(sa["cell"]), -1).any(1))[0]
                bad.append(f"seg {k} differs at {len(idx)} segs first {idx[:4]}")
    h = eng.tm_header(0)
    sc = orc.tm_scalars()
    for k1, k2 in [("lrn_iter", "lrn_iter"), ("iter", "iter"), ("pam_counter", "pam_counter"),
                   ("learned_seq_length", "learned_seq_length"), ("n_inf_pat", "n_prev_inf"),
                   ("n_lrn_pat", "n_prev_lrn"), ("n_upd", "n_updates")]:
        if getattr(h, k1) != sc[k2]:
            bad.append(f"{k1} gpu {getattr(h, k1)} orc {sc[k2]}")
    rs = orc.tm_rng_state()
    if list(h.rng_state) != list(rs[:31]) or h.rng_f != rs[31] or h.rng_r != rs[32]:
        bad.append("tm rng state differs")
    if h.error:
        bad.append(f"error flags {h.error}")
    if bad:
        print(f"[{tag}] MISMATCH:", *bad, sep="\n   ", flush=True)
    return not bad


def cmp_sp(eng, orc, tag):
    a = eng.sp_state(0)
    b = orc.sp_state()
    bad = []
    for k in ["potential", "perm", "connected", "overlap_dc", "active_dc"]:
        if not np.array_equal(a[k], b[k]):
            d = np.argwhere(a[k] != b[k])
            bad.append(f"sp {k} differs at {len(d)} e.g. {d[:3].tolist()}")
    if a["iter"] != b["iter"] or a["iter_learn"] != b["iter_learn"]:
        bad.append(f"sp iters {a['iter']},{a['iter_learn']} vs {b['iter']},{b['iter_learn']}")
    if bad:
        print(f"[{tag}] SP MISMATCH:", *bad, sep="\n   ", flush=True)
    return not bad


def main():
    print("device", torch.cuda.get_device_name(0), flush=True)
    d = np.load(os.path.join(ROOT, "tests/golden/model1_traces.npz"))
    tr = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))]
    t0 = time.time()
    eng = rt.HTMEngine(1, seg_capacity=1 << 16)
    torch.cuda.synchronize()
    print("engine created in %.2fs, %.1f MB" % (time.time() - t0, eng.device_bytes() / 1e6), flush=True)
    eng.set_option(rt._lib.OPT_KEEP_OVERLAPS, 1)
    orc = oracle.OracleModel()
    ok = cmp_sp(eng, orc, "init")
    print("SP init parity:", ok, flush=True)
    v = torch.zeros(1, dtype=torch.float64, device="cuda")
    first_bad = None
    t_gpu = 0.0
    for k in range(N_TRAIN):
        v.fill_(float(tr[k]))
        torch.cuda.synchronize()
        t1 = time.time()
        s = eng.step(v)
        torch.cuda.synchronize()
        t_gpu += time.time() - t1
        so = orc.step(tr[k], True, True)
        ac = eng.get_output("active_columns")[0].cpu().numpy()
        ao = np.zeros(2048, np.uint8)
        ao[orc.active_columns()] = 1
        sg = float(s[0].item())
        if not np.array_equal(ac, ao) or sg != float(so):
            print(f"step {k}: active equal={np.array_equal(ac, ao)} score gpu {sg} orc {so}", flush=True)
            ovg = eng.get_output("sp_overlaps")[0].cpu().numpy()
            ovo = orc.sp_overlaps()
            print("  overlaps equal:", np.array_equal(ovg, ovo), "gpu max", ovg.max(), "orc max", ovo.max(),
                  "ndiff", int((ovg != ovo).sum()), flush=True)
            print("  gpu active", np.nonzero(ac)[0].tolist(), flush=True)
            print("  orc active", np.nonzero(ao)[0].tolist(), flush=True)
            print("  gpu ov at gpu active", ovg[np.nonzero(ac)[0]].tolist(), flush=True)
            first_bad = k
        if k < 5 or k % 50 == 0 or first_bad is not None:
            okt = cmp_state(eng, orc, f"train step {k}")
            if not okt and first_bad is None:
                first_bad = k
        if first_bad is not None:
            cmp_sp(eng, orc, f"step {k}")
            break
    print(f"train: {k + 1} steps, first_bad={first_bad}, gpu step avg {t_gpu / (k + 1) * 1e3:.2f} ms", flush=True)
    if first_bad is None:
        cmp_sp(eng, orc, "after train")
        cmp_state(eng, orc, "after train")
        eng.set_learning(True, False)
        te = d["test_cpu"]
        for frozen in [1]:
            eng.use_frozen_index(bool(frozen))
            bad = None
            for k in range(N_TEST):
                v.fill_(float(te[k]))
                s = eng.step(v)
                so = orc.step(te[k], True, False)
                if float(s[0].item()) != float(so):
                    print(f"test step {k}: score gpu {float(s[0].item())} orc {so}", flush=True)
                    bad = k
                    break
            okt = cmp_state(eng, orc, "after test")
            print(f"test frozen={frozen}: first_bad={bad} state_ok={okt}", flush=True)
    eng.status()
    print("DONE", flush=True)


if __name__ == "__main__":
    main()
