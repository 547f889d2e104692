"""bench.py's multi-rank contract on the GPU box.

``bench.py --gpus 2`` run OUTSIDE torchrun must start the ranks itself (a
child torchrun, no exec) and print ``n_gpus: 2`` with a verified CRC of
every slice of the last fan-out.  The 1-GPU box cannot give RCCL two GPUs,
so the rehearsal uses gloo, whose collectives ShardedLoader stages through
host memory; the RCCL path is the same loader with device tensors.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(tmp_path, *extra):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
           "--window-mib", "64", "--file-gib", "0.25", "--lat-samples", "100",
           "--dir", str(tmp_path), *extra]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_two_ranks_self_launch_gloo(tmp_path):
    out = _run_bench(tmp_path, "--gpus", "2", "--backend", "gloo")
    assert out["n_gpus"] == 2
    assert out["rccl"]["world_size"] == 2
    assert out["rccl"]["allgather_verified"] is True
    assert out["verified_crc32c"] is True
    assert len(out["per_rank"]["load_GiBps_per_rank"]) == 2
    assert out["config"]["parallelism"] == "dp2+allgather"
    # every timed step's gathered shards delivered and slice-checked
    assert out["rccl"]["delivered_steps"] == 2 and out["rccl"]["per_step_slice_check"] is True
    assert out["per_rank"]["delivered_steps_per_rank"] == [2, 2]


@pytest.mark.gpu
def test_bench_single_rank_contract(tmp_path):
    out = _run_bench(tmp_path)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["n_gpus"] == 1 and out["steps"] == 2 and out["warmup"] == 1
    assert out["verified_crc32c"] is True and out["value"] > 0
