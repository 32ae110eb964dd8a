"""bench.py's multi-rank launch on the GPU box: `--gpus 2` spawns two rank processes that
share the one MI355X through the host exchange (RCCL refuses two ranks on one GPU), and the
row-sharded run describes the same problem as one rank:

* strong scaling (default): 2 ranks x N/2 rows == 1 rank x N rows;
* weak scaling: 2 ranks x N rows == 1 rank x 2N rows;

test RMSE per iteration and the free energy agree to summation order (1e-9 relative: only
the per-level sums over rows change order). The 8-GPU RCCL run executes the same per-rank
code with ncclAllReduce as the collective.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REL = 1e-9


def _bench(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "tiny", "--steps", "2",
                          "--warmup", "1", "--no-cpu-baseline"] + list(args),
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout          # rank 0 alone prints
    return json.loads(lines[0])


def _close(a, b):
    assert abs(a - b) <= REL * abs(b), (a, b)


@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_two_rank_bench_matches_one_rank(scaling):
    two = _bench("--gpus", "2", "--transport", "host", "--scaling", scaling)
    assert two["n_gpus"] == 2 and two["n_ranks_seen"] == 2 and two["transport"] == "host"
    assert two["scaling"] == scaling
    rows = 200_000 if scaling == "strong" else 400_000
    assert two["config"]["rows_total"] == rows
    one = _bench("--rows", str(rows))
    assert one["n_gpus"] == 1 and one["config"]["rows_total"] == rows
    assert len(two["test_rmse_trace"]) == len(one["test_rmse_trace"]) == 3
    for a, b in zip(two["test_rmse_trace"], one["test_rmse_trace"]):
        assert abs(a - b) <= 1e-8 * b, (two["test_rmse_trace"], one["test_rmse_trace"])  # 9 digits printed
    _close(two["test_rmse"], one["test_rmse"])
    _close(two["free_energy"], one["free_energy"])
    assert one["test_rmse_trace"][-1] < one["test_rmse_trace"][0]
    assert len(one["rccl_libs"]) <= 1 and len(two["rccl_libs"]) <= 1


def test_eight_rank_bench_matches_one_rank():
    """The driver's N = 8 launch rehearsed on one GPU: `--gpus 8` spawns eight rank processes
    (one per GPU on a node; here they share the card through the host exchange), each owning
    1/8 of the rows (strong scaling), the level schedule max-reduced over the ranks, the
    deferred split sweeps with a per-level all-reduce of 8 shards' statistics -- the same run
    as one rank over all rows."""
    eight = _bench("--gpus", "8", "--transport", "host")
    assert eight["n_gpus"] == 8 and eight["n_ranks_seen"] == 8 and eight["transport"] == "host"
    assert eight["config"]["rows_total"] == 200_000 and eight["config"]["rows_per_gpu"] == 25_000
    assert eight["config"]["parallelism"] == "row-sharded dp8"
    one = _bench("--rows", "200000")
    for a, b in zip(eight["test_rmse_trace"], one["test_rmse_trace"]):
        assert abs(a - b) <= 1e-8 * b, (eight["test_rmse_trace"], one["test_rmse_trace"])
    _close(eight["test_rmse"], one["test_rmse"])
    _close(eight["free_energy"], one["free_energy"])


def test_bench_rank_fault_ends_the_run():
    """The N-rank launch with a faulting rank (VBFM_FAULT=comm on rank 2 of 4: its first exchange
    inside a sweep fails as a failed collective would): that rank exits non-zero and the launcher
    stops the ranks waiting for it in the exchange, well before any deadline; the exchange fields
    of a good run are in the line (host transport: every call timed)."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(VBFM_FAULT="comm", VBFM_FAULT_RANK="2")
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "tiny", "--steps", "2",
                          "--warmup", "1", "--no-cpu-baseline", "--gpus", "4", "--transport", "host"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and not [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert "rank 2/4: w sweep, level 0: VBFM_FAULT=comm" in out.stderr, out.stderr[-3000:]
    # the first rank seen failing: rank 2, or a rank whose exchange failed when rank 2 left
    assert " of 4 exited with status" in out.stderr, out.stderr[-3000:]
    assert time.time() - t0 < 200
    good = _bench("--gpus", "2", "--transport", "host")
    ex = good["exchange"]
    assert good["exchange_bytes"] > 0 and ex["calls_per_step"] > 0 and ex["timed"] > 0 and good["ms_exchange"] > 0
