"""bench.py --gpus N launches its own N ranks when no launcher set
WORLD_SIZE (torch.distributed.run, one process per GPU), refuses a --gpus that
disagrees with WORLD_SIZE, and reports n_gpus / total_streams from the real
world size.  On the CPU: gloo and the stand-in engine (tests/bench_standin.py);
the GPU path differs only in the engine and the RCCL backend."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    return env


def test_bench_gpus_2_launches_two_ranks():
    S = 8
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-standin", "--steps", "6",
           "--warmup", "2", "--condition", "2", "--other-steps", "4", "--streams", str(S)]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints the one line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["total_streams"] == 2 * S and out["config"]["streams_per_gpu"] == S
    assert out["steps"] == 6 and out["value"] > 0
    assert "STAND-IN" in out["data"]
    assert out["run_mode"]["steps"] == 4
    assert "launching 2 ranks" in r.stderr


def test_bench_refuses_gpus_disagreeing_with_world_size():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--cpu-standin", "--steps", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "disagrees with WORLD_SIZE=2" in r.stderr


def test_standin_scores_are_a_function_of_the_global_stream():
    import torch
    from bench_standin import StandInEngine, standin_score
    e = StandInEngine(4, 10)
    out = torch.empty(4, dtype=torch.float32)
    e.step(torch.tensor([3.0, 4.0, 5.0, 6.0], dtype=torch.float64), out)
    want = np.array([standin_score(10 + i, 3 + i) for i in range(4)], np.float32)
    assert np.array_equal(out.numpy(), want)


def test_config5_inputs_follow_the_aggregate_schema():
    """bench.py's config-5 workload (no GPU): the four aggregate fields in the
    MultiEncoder's sorted order (cpu, max, mean, mem), each stream's records
    the reference's TestingData aggregates shifted by 97 records, cpu/mem
    jittered and clipped to [0, 100], response times scaled per stream; a
    stream's shard of the inputs equals the same streams of the whole; the
    training rows skip records with a null field (ModelTraining.py:29-32)."""
    import bench
    d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
    assert [f[0] for f in bench.FIELDS5] == sorted(f[0] for f in bench.FIELDS5)
    rec, mean, viol = bench.config5_inputs(d, 8, 0, 8, 12)
    assert rec.shape == (12, 8, 4) and mean.shape == (12, 8) and viol.shape == (12, 8)
    assert np.all((rec[..., 0] >= 0) & (rec[..., 0] <= 100) & (rec[..., 3] >= 0) & (rec[..., 3] <= 100))
    idx = (np.arange(12)[:, None] + 97 * np.arange(8)[None, :]) % len(d["test_cpu"])
    assert np.all(np.abs(rec[..., 0] - d["test_cpu"][idx]) <= 2 + 1e-9)
    np.testing.assert_array_equal(rec[..., 2], mean)
    np.testing.assert_array_equal(viol, d["test_violations"][idx])
    part, _, _ = bench.config5_inputs(d, 8, 3, 6, 12)
    np.testing.assert_array_equal(part, rec[:, 3:6])
    tr = bench.config5_train_values(d)
    assert tr.shape[1] == 4 and len(tr) <= 2184 and not np.isnan(tr).any()
