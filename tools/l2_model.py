#!/usr/bin/env python3
"""The Fourier search's L2-miss traffic, modelled from its own workgroup timeline.

Input: the diagnostic build's per-workgroup stamps of one C3 launch (tools/clock_stamp.py --dump):
s_memrealtime at the loop's start and end, the XCC the workgroup ran on, and its work item's tile
range.  Each workgroup is taken to stream its tiles at a constant rate between its two stamps
(stage k of K at t0 + (t1 − t0)·k/K); per XCC the reads are replayed in time order through an LRU
cache of the L2's 4 MiB at tile granularity (5 KiB of A fragments + 256 B of row constants per
tile), each workgroup first reading its 8 range blocks' fragments (6 KiB each, never shared: the
4 workgroups of a block group run on 4 different XCCs).  The misses × bytes is the model's
fabric read traffic, to set beside the corrected FETCH_SIZE (TCC_EA0_RDREQ_128B × 128 B).

Printed beside it: the lockstep ("generation") model — every resident set of 64 workgroups per XCC
streams its split together, one miss per tile per generation — which is what the counter would
read if the workgroups of a generation never drifted apart.
usage: tools/l2_model.py STAMPS.npy [--l2-mib 4] [--blocks-per-wg 8]"""
import collections
import json
import sys

import numpy as np

path = sys.argv[1]
l2_mib = float(sys.argv[sys.argv.index("--l2-mib") + 1]) if "--l2-mib" in sys.argv else 4.0
bpw = int(sys.argv[sys.argv.index("--blocks-per-wg") + 1]) if "--blocks-per-wg" in sys.argv else 8
TILE_B = 5 * 64 * 16 + 16 * 16  # KS = 5 A fragments (1 KiB each) + the tile's kDftCS = 16 uint4 of row constants
RFRAG_B = 6 * 64 * 16  # six B fragments of one range block
STAGE = 4  # tiles per LDS stage

raw = np.load(path)
rt0, rt1 = raw[:, 2].astype(np.float64), raw[:, 3].astype(np.float64)
xcc = (raw[:, 4] >> 32).astype(np.int64) & 0xF
z, w = (raw[:, 5] & 0xFFFFFFFF).astype(np.int64), (raw[:, 5] >> 32).astype(np.int64)
nwg = len(raw)
cap_tiles = int(l2_mib * 2**20 // TILE_B)

def lru_misses(t_start, t_end):
    """Tile misses per XCC of the workgroups' reads replayed through an LRU of cap_tiles."""
    ev_t, ev_x, ev_tile, ev_n = [], [], [], []
    for g in range(nwg):
        nt = int(w[g] - z[g])
        if nt <= 0:
            continue
        ns = (nt + STAGE - 1) // STAGE
        k = np.arange(ns)
        ev_t.append(t_start[g] + (t_end[g] - t_start[g]) * k / ns)
        ev_x.append(np.full(ns, xcc[g]))
        ev_tile.append(z[g] + STAGE * k)
        ev_n.append(np.minimum(STAGE, nt - STAGE * k))
    ev_t, ev_x = np.concatenate(ev_t), np.concatenate(ev_x)
    ev_tile, ev_n = np.concatenate(ev_tile), np.concatenate(ev_n)
    out = {}
    for x in np.unique(ev_x):
        sel = np.nonzero(ev_x == x)[0]
        order = sel[np.argsort(ev_t[sel], kind="stable")]
        lru = collections.OrderedDict()
        m = 0
        for e in order:
            t0 = int(ev_tile[e])
            for t in range(t0, t0 + int(ev_n[e])):
                if t in lru:
                    lru.move_to_end(t)
                else:
                    m += 1
                    lru[t] = None
                    if len(lru) > cap_tiles:
                        lru.popitem(last=False)
        out[int(x)] = m
    return out


per_xcc = lru_misses(rt0, rt1)
miss_tiles = sum(per_xcc.values())
# the same replay on a lockstep timeline: per XCC, the workgroups in start order in generations of 64,
# each generation starting together when the previous one ends (every loop the median duration)
med = float(np.median(rt1 - rt0))
ls0 = np.zeros(nwg)
for x in np.unique(xcc):
    gs = np.nonzero(xcc == x)[0]
    gs = gs[np.argsort(rt0[gs], kind="stable")]
    ls0[gs] = (np.arange(len(gs)) // 64) * med
lock_lru = sum(lru_misses(ls0, ls0 + med).values())
model_b = miss_tiles * TILE_B + nwg * bpw * RFRAG_B
# lockstep: per XCC, generations of (resident) workgroups each read their splits' distinct tiles once
resident = 64  # 32 CUs × 2 workgroups (108 VGPRs: 4 waves per SIMD; 8-wave workgroups)
lock_tiles = 0
for x in np.unique(xcc):
    gs = np.nonzero(xcc == x)[0]
    gs = gs[np.argsort(rt0[gs], kind="stable")]
    for i in range(0, len(gs), resident):
        grp = gs[i:i + resident]
        tiles = set()
        for g in grp:
            tiles.update(range(int(z[g]), int(w[g])))
        lock_tiles += len(tiles)
lock_b = lock_tiles * TILE_B + nwg * bpw * RFRAG_B
span = (rt1.max() - rt0.min()) / 100.0  # µs (100 MHz s_memrealtime)
dur = (rt1 - rt0) / 100.0
print(json.dumps({"stamps": path, "workgroups": nwg, "xcc_count": int(len(np.unique(xcc))),
                  "l2_mib": l2_mib, "cap_tiles": cap_tiles, "launch_span_us": round(float(span), 1),
                  "wg_loop_us": {"p10": round(float(np.percentile(dur, 10)), 1),
                                 "median": round(float(np.median(dur)), 1),
                                 "p90": round(float(np.percentile(dur, 90)), 1)},
                  "timeline_lru_model_bytes": int(model_b), "timeline_lru_miss_tiles_per_xcc": per_xcc,
                  "lockstep_model_bytes": int(lock_b),
                  "lockstep_timeline_lru_bytes": int(lock_lru * TILE_B + nwg * bpw * RFRAG_B)}, indent=1))
