"""HBM traffic per dispatch from rocprofv3 --pmc passes, calibrated.

Usage: python tools/pmc_summary.py <run dir> <out dir> [--calib <calib dir> <calib bytes json>]

<run dir> holds the rocprofv3 output directories of the passes over ONE
command (tools/gpu_prof.sh):
  pmc_rd/     TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
  pmc_fetch/  FETCH_SIZE
  pmc_wr/     WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
  pmc_l2/     TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum (optional: fleets, whose shared model is L2-served)
  pmc_sq1/, pmc_sq2/  SQ counters (optional): issue / wait fractions of the waves' cycles
  prof/       --kernel-trace --stats (kernel_stats.csv is copied along)
Counters are per dispatch; the median over the dispatches of each kernel is
reported.  Read bytes are counted from the L2 memory-side read requests by
size class, 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B, write bytes
as 64 x WRREQ_64B + 32 x (WRREQ - WRREQ_64B); FETCH_SIZE / WRITE_SIZE are
reported beside them.  MI355X_MICROARCH.md (HBM section) calibrates
FETCH_SIZE only for 16-byte-per-lane streaming reads (it reports half of
them); --calib checks the request-size formula and FETCH_SIZE against the
known bytes of tools/fetch_calib's access patterns (the widths the frozen TM
kernel issues), and the verdict is written beside the numbers.

Output <out dir>/pmc_summary.json: {"kernels": {name: {... ,
"hbm_bytes_per_dispatch": B, "formula": "..."}}, "calibration": {...}} --
the file bench.py --pmc-summary reads.
"""
import csv
import json
import os
import shutil
import statistics
import sys


def load_pass(path):
    """{kernel: {counter: [values per dispatch]}}"""
    f = os.path.join(path, "run_counter_collection.csv")
    out = {}
    if not os.path.exists(f):
        return out
    for r in csv.DictReader(open(f)):
        out.setdefault(r["Kernel_Name"], {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return out


def med(d, k, c):
    v = d.get(k, {}).get(c)
    return statistics.median(v) if v else None


# SQ passes (8 SQ counters each): where the waves' cycles go.  SQ_WAVE_CYCLES,
# SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles summed over waves;
# WAIT_ANY (parked on s_waitcnt / s_barrier) + WAIT_INST_ANY (ready, not
# issued) + ACTIVE_INST_ANY (issuing) ~= WAVE_CYCLES (MI355X_MICROARCH.md,
# rocprofv3 PMC slots).
SQ_PASSES = ("pmc_sq1", "pmc_sq2", "pmc_sq3")


def sq_summary(sq, k):
    """Fractions of the waves' cycles (median per dispatch) from the SQ passes;
    each counter is divided by SQ_WAVE_CYCLES of its own pass (every SQ pass
    collects it)."""
    def g(c):
        for d in sq:
            v = med(d, k, c)
            if v is not None:
                return v
        return None

    def frac(c):
        for d in sq:
            v, w = med(d, k, c), med(d, k, "SQ_WAVE_CYCLES")
            if v is not None and w:
                return round(v / w, 4)
        return None
    wc = g("SQ_WAVE_CYCLES")
    if not wc:
        return None
    out = {"waves": g("SQ_WAVES"), "wave_cycles": wc, "busy_cycles": g("SQ_BUSY_CYCLES")}
    for name, c in (("issue_active", "SQ_ACTIVE_INST_ANY"), ("waiting", "SQ_WAIT_ANY"),
                    ("issue_stalled", "SQ_WAIT_INST_ANY"), ("valu", "SQ_ACTIVE_INST_VALU"),
                    ("salu", "SQ_ACTIVE_INST_SCA"), ("lds", "SQ_ACTIVE_INST_LDS"),
                    ("vmem", "SQ_ACTIVE_INST_VMEM"), ("flat", "SQ_ACTIVE_INST_FLAT"),
                    ("misc", "SQ_ACTIVE_INST_MISC"), ("lds_issue_stalled", "SQ_WAIT_INST_LDS")):
        v = frac(c)
        if v is not None:
            out[name] = v
    bc, la = g("SQ_LDS_BANK_CONFLICT"), g("SQ_LDS_IDX_ACTIVE")
    if bc is not None and la:
        out["lds_bank_conflict_over_lds_active"] = round(bc / la, 4)
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM", "SQ_INSTS_FLAT",
              "SQ_INSTS_BRANCH", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INST_LEVEL_VMEM",
              "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
        v = g(c)
        if v is not None:
            out.setdefault("counts", {})[c] = v
    if out.get("waves"):
        out["cycles_per_wave"] = round(4 * wc / out["waves"], 1)  # quad-cycles -> shader cycles
    out["note"] = ("fractions of SQ_WAVE_CYCLES (median per dispatch): issue_active = ACTIVE_INST_ANY, "
                   "waiting = WAIT_ANY (s_waitcnt on memory/LDS or s_barrier), issue_stalled = WAIT_INST_ANY; "
                   "per-unit issue fractions (valu, salu, lds, vmem, flat) overlap")
    return out


def summarise(run):
    rd, fe, wr, l2 = (load_pass(os.path.join(run, p)) for p in ("pmc_rd", "pmc_fetch", "pmc_wr", "pmc_l2"))
    sq = [load_pass(os.path.join(run, p)) for p in SQ_PASSES]
    kernels = {}
    for k in set(rd) | set(fe) | set(wr) | set(l2) | set().union(*sq):
        e = {}
        sqs = sq_summary(sq, k)
        if sqs:
            e["sq"] = sqs
        hit, miss, req = (med(l2, k, c) for c in ("TCC_HIT_sum", "TCC_MISS_sum", "TCC_REQ_sum"))
        if None not in (hit, miss):
            e["l2"] = {"hit": hit, "miss": miss, "req": req,
                       "hit_rate": round(hit / (hit + miss), 4) if hit + miss > 0 else None}
        r32, r64, r128, rall = (med(rd, k, c) for c in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum",
                                                       "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_sum"))
        w64, wall = med(wr, k, "TCC_EA0_WRREQ_64B_sum"), med(wr, k, "TCC_EA0_WRREQ_sum")
        if None not in (r32, r64, r128):
            e["read_bytes"] = 32 * r32 + 64 * r64 + 128 * r128
            e["rdreq"] = {"all": rall, "32B": r32, "64B": r64, "128B": r128}
        if None not in (w64, wall):
            e["write_bytes"] = 64 * w64 + 32 * (wall - w64)
            e["wrreq"] = {"all": wall, "64B": w64}
        fs, ws = med(fe, k, "FETCH_SIZE"), med(wr, k, "WRITE_SIZE")
        if fs is not None:
            e["fetch_size_bytes"] = fs * 1024
        if ws is not None:
            e["write_size_bytes"] = ws * 1024
        n = max(len(d.get(k, {}).get(c, [])) for d, c in ((rd, "TCC_EA0_RDREQ_sum"), (fe, "FETCH_SIZE"),
                                                         (wr, "WRITE_SIZE"), *((x, "SQ_WAVE_CYCLES") for x in sq)))
        e["dispatches"] = n
        if "read_bytes" in e and "write_bytes" in e:
            e["hbm_bytes_per_dispatch"] = e["read_bytes"] + e["write_bytes"]
            e["formula"] = ("median per dispatch of 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B + "
                            "64*WRREQ_64B + 32*(WRREQ - WRREQ_64B) (TCC_EA0 memory-side requests)")
        kernels[k] = e
    return kernels


def main():
    run, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    out = {"source": run, "kernels": summarise(run)}
    if "--calib" in sys.argv:
        i = sys.argv.index("--calib")
        cdir, cjson = sys.argv[i + 1], sys.argv[i + 2]
        known = json.load(open(cjson))
        ck = summarise(cdir)
        cal = {}
        for name, kb in known.items():
            m = [v for k, v in ck.items() if k.startswith(name + "(") or k == name]
            if not m:
                continue
            e = m[0]
            row = {"known": kb}
            if "read" in kb:
                row["formula_over_known"] = round(e.get("read_bytes", 0) / kb["read"], 4)
                row["fetch_size_over_known"] = round(e.get("fetch_size_bytes", 0) / kb["read"], 4)
                row["rdreq"] = e.get("rdreq")
            else:
                row["formula_over_known"] = round(e.get("write_bytes", 0) / kb["write"], 4)
                row["write_size_over_known"] = round(e.get("write_size_bytes", 0) / kb["write"], 4)
                row["wrreq"] = e.get("wrreq")
            cal[name] = row
        out["calibration"] = {"source": cdir, "patterns": cal,
                              "note": "random gathers move whole lines: their formula/known is the line "
                                      "over-fetch of the pattern, not a counter error; streaming patterns "
                                      "(stream16, stream4, runs16, wstream16) check the counters"}
    json.dump(out, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    ks = os.path.join(run, "prof", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, "kernel_stats.csv"))
    top = {k: {x: v.get(x) for x in ("hbm_bytes_per_dispatch", "fetch_size_bytes", "write_size_bytes")}
           for k, v in out["kernels"].items() if "htm_run" in k or "tm_step" in k}
    print(json.dumps({"kernels": top, "calibration": out.get("calibration", {}).get("patterns")}, indent=1))


if __name__ == "__main__":
    main()
