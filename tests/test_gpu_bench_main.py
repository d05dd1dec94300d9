"""bench.py's own main() at N = 2 with the HIP engine (the code the driver's 8-GPU run
executes): two ranks launched by bench.py itself (torch.distributed.run), both on the one GPU of this box,
over `gloo` (RCCL takes one rank per GPU) — the frame in row stripes + all-gather, each rank's resolve
writing its shard's tuples into the all-gather buffer or the node-shared pinned buffer (two processes
registering one mapping), the other exchange, the device-resident, stream and C5 legs, HIP-event phase
clocks, the MAX over ranks.  The two-rank records equal the one-rank run's byte for byte, and every leg's
check holds.  Reference parallelism replaced: encode/EncodingEngine2.hpp:118-171."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--size", "512", "--steps", "2", "--warmup", "1", "--side-steps", "1", "--cpu-budget", "0", "--alt-steps",
        "0", "--drop-in", "0"]


def _bench(tmp_path, name, *extra):
    out = str(tmp_path / f"{name}.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *ARGS, *extra, "--out", out],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    return json.load(open(out))


@pytest.fixture(scope="module")
def one_rank(tmp_path_factory):
    return _bench(tmp_path_factory.mktemp("w1"), "w1", "--gpus", "1")


@pytest.mark.parametrize("tuples", ["gather", "node"])
def test_bench_main_two_ranks_on_one_gpu(tmp_path, one_rank, tuples):
    shm = {f for f in os.listdir("/dev/shm") if f.startswith("fracenc_tuples_")}
    line = _bench(tmp_path, "w2", "--gpus", "2", "--backend", "gloo", "--share-gpu", "--tuples", tuples)
    assert {f for f in os.listdir("/dev/shm") if f.startswith("fracenc_tuples_")} == shm
    rec, want = line["records"], one_rank["records"]
    assert rec["tuples_sha16"] == want["tuples_sha16"] and rec["n"] == want["n"] == 4096
    other = "node" if tuples == "gather" else "gather"
    assert rec["own_slice_in_gather"] and rec["device_leg_equals_e2e"] and rec[f"{other}_equals_headline"]
    assert line["tuples_out"] == tuples and line[f"{other}_value"]["value"] > 0
    assert line["c5"]["records"] == one_rank["c5"]["records"]
    assert line["n_gpus"] == 2 and line["ms_per_step"] == max(line["rank_ms_per_step"])
    assert line["config"]["engine"] == "mfma" and line["search_form"] == "fourier"
    for k, v in line["phases_ms"].items():
        assert v == max(r[k] for r in line["phases_ms_by_rank"]), k
    assert all(r["frame_allgather"] > 0 and r["search"] > 0 for r in line["phases_ms_by_rank"])
    assert one_rank["records"]["own_slice_in_gather"] and one_rank["records"]["device_leg_equals_e2e"]


@pytest.mark.parametrize("tuples", ["node", "gather"])
def test_bench_main_rccl_group_at_world_one(tmp_path, one_rank, tuples):
    """bench.py under torch.distributed.run with one rank and --group: the nccl (RCCL) process group on the GPU
    and every N > 1 path the driver's 8-GPU line runs — frame stripes + RCCL all-gather, the RCCL tuple
    all-gather and the node buffer's RCCL token, the float64 all-reduce / all-gather of the clocks, C5's
    all-gathers — with the records equal to the plain one-rank run's."""
    import bench

    out = str(tmp_path / f"group_{tuples}.json")
    rc = bench.launch_ranks(1, script=os.path.join(ROOT, "bench.py"),
                            argv=[*ARGS, "--gpus", "1", "--group", "--tuples", tuples, "--out", out])
    assert rc == 0
    line = json.load(open(out))
    rec, want = line["records"], one_rank["records"]
    other = "node" if tuples == "gather" else "gather"
    assert rec["tuples_sha16"] == want["tuples_sha16"] and rec["n"] == want["n"]
    assert rec["own_slice_in_gather"] and rec["device_leg_equals_e2e"] and rec[f"{other}_equals_headline"]
    assert line["tuples_out"] == tuples and line[f"{other}_value"]["value"] > 0
    assert line["c5"]["records"] == one_rank["c5"]["records"]
    assert line["phases_ms"]["frame_allgather"] > 0 and line["search_form"] == "fourier"
