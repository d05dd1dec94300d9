"""bench.py's N > 1 orchestration, executed on the CPU: bench.launch_ranks
starts `gloo` ranks under torch.distributed.run; each runs bench.FrameStep (frame upload, search of
its shard, tuples into the node's shared buffer or the all-gather buffer + all-gather, tuples out) with the oracle
stand-in engine, the same timed() bracket and headline_fields() the GPU headline uses.  No scaling
curve is measured here: only the orchestration's correctness (records, MAX over ranks, exit
status).  Reference parallelism being replaced: EncodingEngineCore2's thread pool over range items
(encode/EncodingEngine2.hpp:118-171)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SCRIPT = os.path.join(HERE, "bench_rank_cpu.py")
STEPS = 2


def _run(tmp_path, world, fail_rank=None, tuples="node"):
    import bench

    out = str(tmp_path / f"line_{world}.json")
    argv = [out, str(STEPS)] + ([] if fail_rank is None else [str(fail_rank)])
    env = dict(os.environ, OMP_NUM_THREADS="1", BENCH_TUPLES=tuples)
    if world == 1:  # a single rank without a process group, as bench.py runs at N = 1
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


@pytest.mark.parametrize("world,tuples", [(2, "node"), (3, "node"), (4, "node"), (8, "node"), (3, "gather"),
                                          (8, "gather")])
def test_bench_orchestration_on_gloo_ranks(tmp_path, single, oracle, world, tuples):
    import bench
    import fractencode_amd as F
    from fractencode_amd.distributed import records_from_tuples

    before = _node_files()
    rc, out = _run(tmp_path, world, tuples=tuples)
    assert rc == 0
    assert _node_files() == before  # the shared tuple buffer's file is gone once every rank mapped it
    d = json.load(open(out))
    line = d["line"]
    # the gathered records equal the single-rank run's, byte for byte, and the reference's (oracle); the
    # frame reached every rank as row stripes and one all-gather (64 rows: uneven stripes at world 3); the
    # tuples met in the node's shared host buffer, or through the all-gather
    assert d["stripes"] and not single["stripes"]
    assert d["node"] == (tuples == "node") and not single["node"]
    assert d["digest"] == single["digest"] and d["tuples"] == single["tuples"]
    tuples = np.frombuffer(bytes.fromhex(d["tuples"]), dtype=F.TUPLE)
    assert len(tuples) == 93
    rng = np.random.default_rng(3)
    plane = rng.integers(0, 256, (64, 96), dtype=np.uint8)
    doms = F.create_uniform_grid(96, 64, 16, 8)
    rngs = F.create_uniform_grid(96, 64, 8, 8)[:93]
    rec = records_from_tuples(tuples, rngs, doms)
    want, _, _ = oracle.estimate(plane, oracle.uniform_grid(96, 64, 16, 8), oracle.uniform_grid(96, 64, 8, 8)[:93])
    for a, b in (("dx", "dx"), ("dy", "dy"), ("transform", "t"), ("distance", "dist"), ("contrast", "s"),
                 ("brightness", "o")):
        np.testing.assert_array_equal(rec[a], want[b], err_msg=a)
    # every rank's slice of the gather is its own shard
    ranks = d["ranks"]
    assert sorted(r for r, _, _ in ranks) == list(range(world)) and all(ok for _, _, ok in ranks)
    # n_gpus, value and ms_per_step come from the slowest rank's time
    slowest = max(t for _, t, _ in ranks)
    assert line["n_gpus"] == world and line["steps"] == STEPS
    assert line["ms_per_step"] == round(1e3 * slowest / STEPS, 3)
    assert line["value"] == round(93 / (slowest / STEPS), 1)
    assert line["metric"] == bench.METRIC and line["unit"] == "range-blocks/s" and line["scaling"] == "strong"


def test_launch_ranks_returns_the_childrens_status(tmp_path):
    rc, _ = _run(tmp_path, 2, fail_rank=1)
    assert rc != 0
