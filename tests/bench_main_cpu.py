"""bench.py's own main() on the CPU (test infrastructure, launched by tests/test_bench_ranks.py through
bench.launch_ranks → torch.distributed.run, or run directly for world size 1): the same main() the GPU
headline runs, given the oracle stand-in engine (tests/oracle_engine.py), the `gloo` backend in place of
RCCL and CPU devices.  FAIL_RANK=r makes rank r exit with status 3 before main() (the launcher must
report it).
usage: [FAIL_RANK=r] python tests/bench_main_cpu.py <bench.py arguments>"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import bench  # noqa: E402
from oracle_engine import OracleEngine  # noqa: E402

if int(os.environ.get("RANK", "0")) == int(os.environ.get("FAIL_RANK", "-1")):
    sys.exit(3)
bench.main(bench.parse(sys.argv[1:]), engine_factory=OracleEngine.factory, backend="gloo", cuda=False)
