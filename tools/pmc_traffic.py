#!/usr/bin/env python3
"""Writes profiles/pmc_search.json's FORM entry from rocprofv3 --pmc passes (separate runs) over the
same program: fabric read bytes per search launch from the sized read-request counters, write bytes
from WRITE_SIZE, and FETCH_SIZE beside them with the factor between the two.

Read bytes = 32·TCC_EA0_RDREQ_32B + 64·TCC_EA0_RDREQ_64B + 128·TCC_EA0_RDREQ_128B (sums over the
XCDs' L2 channels).  rocprofv3's FETCH_SIZE tallies every request above 32 B at 64 B, so on gfx950
it reads half the bytes of the 128-byte requests a 16-B-per-lane streaming read makes
(MI355X_MICROARCH.md §HBM; calibrated on this kernel's own access pattern by tools/fetch_calib.hip:
1 GiB read once = 8,388,608 128-B requests, FETCH_SIZE 524,288 kB).  The counters see the L2's
misses to the fabric; Infinity Cache hits are among them.
usage: tools/pmc_traffic.py FORM KERNEL_PREFIX RDREQ_CSV FETCH_CSV WRITE_CSV SOURCE_NOTE"""
import csv
import json
import os
import sys

form, prefix, rcsv, fcsv, wcsv, note = sys.argv[1:7]


def per_dispatch(path):
    tot, disp = {}, set()
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].startswith(prefix):
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
    n = max(1, len(disp))
    return {k: v / n for k, v in tot.items()}, len(disp)


rq, nr = per_dispatch(rcsv)
fe, nf = per_dispatch(fcsv)
wr, nw = per_dispatch(wcsv)
n32, n64, n128 = (rq.get(f"TCC_EA0_RDREQ_{s}B_sum", 0.0) for s in (32, 64, 128))
read_b = 32 * n32 + 64 * n64 + 128 * n128
fetch_kb, write_kb = fe.get("FETCH_SIZE", 0.0), wr.get("WRITE_SIZE", 0.0)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = os.path.join(ROOT, "profiles", "pmc_search.json")
d = json.load(open(path)) if os.path.exists(path) else {}
d["_doc"] = ("Fabric-side bytes per search launch (rocprofv3 --pmc, separate passes): reads from the sized L2 "
             "read-request counters, 32·RDREQ_32B + 64·RDREQ_64B + 128·RDREQ_128B; writes from WRITE_SIZE (kB). "
             "FETCH_SIZE is kept beside them: it tallies a 128-B request at 64 B, so it reads half of a 16-B/lane "
             "streaming read on gfx950 (MI355X_MICROARCH.md §HBM; calibrated on this kernel's access pattern by "
             "tools/fetch_calib.hip, profiles/r04/traffic/). Keyed by frac_stats.search_form and the build's "
             "source id.")
sys.path.insert(0, ROOT)
from fractencode_amd import source_id  # noqa: E402

d[form] = {"kernel": prefix, "source_id": source_id(), "dispatches": [nr, nf, nw],
           "rdreq_32b": round(n32, 1), "rdreq_64b": round(n64, 1), "rdreq_128b": round(n128, 1),
           "read_bytes": int(round(read_b)), "fetch_size_kb": round(fetch_kb, 1),
           "fetch_size_to_bytes": round(read_b / (fetch_kb * 1024), 4) if fetch_kb else None,
           "write_size_kb": round(write_kb, 1),
           "correction": "reads from the sized request counters (128-B requests at 128 B); FETCH_SIZE x2 agrees "
                         "within the 64-B requests' share",
           "hbm_bytes_per_launch": int(round(read_b + write_kb * 1024)), "source": note}
json.dump(d, open(path, "w"), indent=1)
print(json.dumps(d[form]))
