"""bench.py's own main() at N > 1, executed on the CPU: bench.launch_ranks starts
`gloo` ranks under torch.distributed.run; each runs bench.main — the headline FrameStep (frame in row
stripes + all-gather, search of its shard, the tuple all-gather or the node-shared buffer), the other
tuple exchange, the device-resident, stream and C5 legs, the per-phase clock, the MAX over ranks and the
line — with the oracle stand-in engine (tests/bench_main_cpu.py).  No scaling curve is measured here:
only the orchestration's correctness (records equal across world sizes, the slowest rank's time, exit
status, nothing left in /dev/shm).  Reference parallelism being replaced: EncodingEngineCore2's thread
pool over range items (encode/EncodingEngine2.hpp:118-171)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SCRIPT = os.path.join(HERE, "bench_main_cpu.py")
SIZE = 64  # 64 ranges, 49 domains; C5: 64 + 16 + 16 ranges
STEPS = 2


def _run(tmp_path, world, tuples="gather", fail_rank=None, group=False):
    import bench

    out = str(tmp_path / f"line_{world}_{tuples}{'_group' if group else ''}.json")
    argv = ["--gpus", str(world), "--size", str(SIZE), "--steps", str(STEPS), "--warmup", "1", "--side-steps", "1",
            "--cpu-budget", "0", "--tuples", tuples, "--out", out] + (["--group"] if group else [])
    env = dict(os.environ, OMP_NUM_THREADS="1")
    if fail_rank is not None:
        env["FAIL_RANK"] = str(fail_rank)
    if world == 1 and group:  # no launcher: bench.py sets up the one-rank group itself
        env = {k: v for k, v in env.items() if k not in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE")}
        rc = subprocess.call([sys.executable, SCRIPT, *argv], env=env)
    elif world == 1:  # a single rank without a process group, as bench.py runs at N = 1
        rc = subprocess.call([sys.executable, SCRIPT, *argv], env=env)
    else:
        rc = bench.launch_ranks(world, script=SCRIPT, argv=argv, env=env)
    return rc, out


@pytest.fixture(scope="module")
def single(tmp_path_factory):
    rc, out = _run(tmp_path_factory.mktemp("w1"), 1)
    assert rc == 0
    return json.load(open(out))


def _node_files():
    return {f for f in os.listdir("/dev/shm") if f.startswith("fracenc_tuples_")}


def test_single_rank_line_is_the_oracles(single, oracle):
    """World 1: the line's records are the reference's (oracle) tuples of every range; the legs agree."""
    import bench
    import fractencode_amd as F
    from fractencode_amd.synth import value_noise
    from oracle_engine import OracleEngine

    frame = value_noise(SIZE, SIZE, 1234)
    e = OracleEngine(frame, F.create_uniform_grid(SIZE, SIZE, 16, 8))
    e.set_ranges(F.create_uniform_grid(SIZE, SIZE, 8, 8))
    e.run()
    want = e.fetch_tuples().tobytes()
    rec = single["records"]
    assert rec["tuples_sha16"] == bench.digest(want) and rec["n"] == SIZE * SIZE // 64
    assert rec["own_slice_in_gather"] and rec["device_leg_equals_e2e"]
    assert single["n_gpus"] == 1 and single["tuples_out"] == "sink"
    assert single["rank_ms_per_step"] == [single["ms_per_step"]]
    assert "gather_value" not in single and "node_value" not in single
    assert single["c5"]["records"]["n"] == SIZE * SIZE // 64 + 2 * (SIZE // 2) ** 2 // 64
    for k in ("device_value", "stream_value"):
        assert single[k]["value"] > 0


@pytest.mark.parametrize("world,tuples", [(2, "gather"), (3, "gather"), (8, "gather"), (2, "node"), (3, "node"),
                                          (8, "node")])
def test_bench_main_on_gloo_ranks(tmp_path, single, world, tuples):
    import bench

    before = _node_files()
    rc, out = _run(tmp_path, world, tuples)
    assert rc == 0
    assert _node_files() == before  # the shared tuple buffers' files are gone once every rank mapped them
    line = json.load(open(out))
    # the gathered records equal the single-rank run's, byte for byte, on every leg; the frame reached every
    # rank as row stripes + one all-gather (64 rows: uneven stripes at world 3)
    rec = line["records"]
    assert rec["tuples_sha16"] == single["records"]["tuples_sha16"]
    assert rec["own_slice_in_gather"] and rec["device_leg_equals_e2e"]
    other = "node" if tuples == "gather" else "gather"
    assert line["tuples_out"] == tuples
    assert rec[f"{other}_equals_headline"] and line[f"{other}_value"]["value"] > 0
    assert line["c5"]["records"] == single["c5"]["records"]
    # n_gpus, value and ms_per_step come from the slowest rank's time
    ranks = line["rank_ms_per_step"]
    assert len(ranks) == world and line["n_gpus"] == world and line["steps"] == STEPS
    assert line["ms_per_step"] == max(ranks)
    n = SIZE * SIZE // 64
    assert abs(line["value"] - n / (line["ms_per_step"] * 1e-3)) <= 1e-3 * line["value"] + 0.1
    assert line["metric"] == bench.METRIC and line["unit"] == "range-blocks/s" and line["scaling"] == "strong"
    # the per-phase breakdown: every rank's, and the maximum over ranks per phase
    by = line["phases_ms_by_rank"]
    assert len(by) == world
    for k, v in line["phases_ms"].items():
        assert v == max(r[k] for r in by), k
    assert all(r["frame_allgather"] > 0 and r["run"] > 0 and r["tuples"] > 0 for r in by)


@pytest.mark.parametrize("tuples", ["gather", "node"])
def test_group_rehearsal_at_world_one(tmp_path, single, tuples):
    """--group: one rank with a process group takes every N > 1 path (frame stripes + all-gather, the tuple
    exchange and the other one as a side leg, the node buffer, C5's all-gathers) — the rehearsal of the RCCL
    line on a one-GPU box; its records equal the plain single-rank run's."""
    rc, out = _run(tmp_path, 1, tuples, group=True)
    assert rc == 0
    line = json.load(open(out))
    rec = line["records"]
    other = "node" if tuples == "gather" else "gather"
    assert line["n_gpus"] == 1 and line["tuples_out"] == tuples
    assert rec["tuples_sha16"] == single["records"]["tuples_sha16"]
    assert rec["own_slice_in_gather"] and rec["device_leg_equals_e2e"] and rec[f"{other}_equals_headline"]
    assert line["c5"]["records"] == single["c5"]["records"]
    assert line["phases_ms"]["frame_allgather"] > 0


def test_launch_ranks_returns_the_childrens_status(tmp_path):
    rc, _ = _run(tmp_path, 2, fail_rank=1)
    assert rc != 0


def test_node_buffer_creation_failure_reaches_every_rank(tmp_path):
    """Rank 0 cannot create the node buffer's file: every rank raises the same error instead of the others
    waiting forever in the name broadcast."""
    script = tmp_path / "node_fail.py"
    script.write_text(
        "import os, sys, torch, torch.distributed as dist\n"
        f"sys.path.insert(0, {os.path.dirname(HERE)!r})\n"
        "import fractencode_amd.distributed as D\n"
        "dist.init_process_group('gloo')\n"
        "rank = dist.get_rank()\n"
        "real = os.open\n"
        "def bad(path, *a, **k):\n"
        "    if 'fracenc_tuples_' in str(path) and rank == 0: raise OSError(28, 'No space left on device')\n"
        "    return real(path, *a, **k)\n"
        "os.open = bad\n"
        "try:\n"
        "    D.NodeTuples([(0, 4), (4, 8)], rank, torch.device('cpu'))\n"
        "    sys.exit(9)\n"
        "except RuntimeError as exc:\n"
        "    assert 'could not create' in str(exc), exc\n"
        "dist.destroy_process_group()\n")
    import bench

    before = _node_files()
    rc = bench.launch_ranks(2, script=str(script), argv=[], env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert rc == 0
    assert _node_files() == before


def test_drop_in_leg_reports_a_failed_core_run_instead_of_raising():
    """bench.drop_in runs oracle/_ref/core_driver (the reference's core with the HIP engine) in child processes
    after the timed region; without a device every run fails at engine creation (exit 4), and the leg records
    each failure in the line instead of ending the bench."""
    import bench
    import torch

    if not os.path.exists(bench.CORE_DRIVER):
        pytest.skip("oracle/_ref/core_driver not built")
    if torch.cuda.is_available():
        pytest.skip("device present: the GPU bench runs the real leg")
    out = bench.drop_in(np.zeros((64, 64), np.uint8), timeout_s=60)
    assert set(out["runs"]) == {name for name, _, _ in bench.DROP_IN_RUNS}
    assert all("exit 4" in r["error"] for r in out["runs"].values())
