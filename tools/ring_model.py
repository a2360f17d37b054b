"""Count what the xGMI ring costs per step, from the host plans (no GPU): the
records each rank pushes, the ring bytes, the wave-level store instructions,
and the 64-byte memory transactions those instructions touch under the
record-major layout of round 5 (``aos``: word w of record r at r NW + w) and
the word-major layout (``soa``: w nrec + r, ops/csrc/stage_common.h
STSP_XG_SOA), for the fused step (lanes = a block's cells in row order,
``xpush``) and the streaming march (lanes = 64 consecutive columns of a row,
the push map).  Input to the 8-GPU step model in docs/ARCHITECTURE.md.

    python tools/ring_model.py --rows fused:96:2:8:6 fused:96:2:8:8 fused:180:2:8:18 march:720:2:8
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stsphere.models.geometry import CubedSphereGrid  # noqa: E402
from stsphere.parallel.layout import TileLayout  # noqa: E402

SLOT_BITS = 24
NW = 8          # fp64 tagged, stage / march kernels: 4 fields x 2 granules of 8 bytes
NW_FUSED = 5    # fp64 fused step (round 6): 5 granules of a 12-bit tag and 52 payload bits
SEG = 64        # bytes per memory transaction counted


def _segments(recs, peers, nrec, j, layout, nw=NW):
    if layout == "aos":
        addr = (recs * NW + j) * 8          # round 5: record-major, 8 granules
    else:
        addr = (j * nrec + recs) * 8        # word-major, nw granules
    return len(set(zip(peers.tolist(), (addr // SEG).tolist())))


def _count(waves, nrec, nw=NW):
    """waves: list of (recs, peers) per store round (active lanes of one wave
    for one push index k).  Returns instruction and transaction counts, in
    total and for the busiest peer (one xGMI link carries one peer pair):
    tx_aos for round 5's record-major 8-granule records, tx_soa for the
    word-major records of nw granules."""
    out = {"records": 0, "store_instr": 0, "tx_aos": 0, "tx_soa": 0, "nw": nw}
    peer = {}
    for recs, peers in waves:
        if recs.size == 0:
            continue
        out["records"] += int(recs.size)
        out["store_instr"] += nw
        for p in np.unique(peers):
            m = peers == p
            d = peer.setdefault(int(p), {"records": 0, "tx_aos": 0, "tx_soa": 0})
            d["records"] += int(m.sum())
            for j in range(NW):
                d["tx_aos"] += _segments(recs[m], peers[m], nrec, j, "aos")
            for j in range(nw):
                d["tx_soa"] += _segments(recs[m], peers[m], nrec, j, "soa", nw)
        for j in range(NW):
            out["tx_aos"] += _segments(recs, peers, nrec, j, "aos")
        for j in range(nw):
            out["tx_soa"] += _segments(recs, peers, nrec, j, "soa", nw)
    out["peers"] = len(peer)
    out["busiest_peer"] = max(peer.values(), key=lambda d: d["records"]) if peer else None
    return out


def fused_row(N, t, ranks, B):
    from stsphere.ops.fused import FusedExchangePlan
    L = TileLayout(N, t, ranks, ng=2)
    X = FusedExchangePlan(L, CubedSphereGrid(N), B=B, ns=3)
    nrec = X.ring_slots
    per = []
    for r in range(ranks):
        xpush = X.producer(r)[0]                      # [nb, B*B, K]
        nb, BB, K = xpush.shape
        waves = []
        for b in range(nb):
            for w0 in range(0, BB, 64):
                lanes = xpush[b, w0:w0 + 64]
                for k in range(K):
                    c = lanes[:, k]
                    c = c[c >= 0].astype(np.int64)
                    waves.append((c & ((1 << SLOT_BITS) - 1), c >> SLOT_BITS))
        per.append(_count(waves, nrec, NW_FUSED))
    return {"path": "fused", "N": N, "t": t, "ranks": ranks, "B": B, "ring_records_per_slot": nrec}, per


def march_row(N, t, ranks):
    from stsphere.ops.xgmi import XgmiPlan, _side_cell
    L = TileLayout(N, t, ranks, ng=2)
    per, nrec = [], 0
    for r in range(ranks):
        xp = XgmiPlan(L, r, 64, 8, 2)
        nrec = xp.ring_slots
        push = xp.push.astype(np.int64)              # [T, 4, g, n]: -2 - code for remote ghosts
        T, _, g, n = push.shape
        lanes = {}
        for li, s, kk, pp in zip(*np.nonzero(push <= -2)):
            i, j = _side_cell(np.array([s]), np.array([kk]), np.array([pp]), n)
            code = -2 - int(push[li, s, kk, pp])
            # the march: a wave's lanes are 60 output columns of one row; a cell
            # pushes its (up to 4) codes in side order
            lanes.setdefault((int(li), int(j[0]), int(i[0]) // 60, int(s)), []).append(code)
        waves = []
        for key, codes in lanes.items():
            c = np.asarray(codes, dtype=np.int64)
            waves.append((c & ((1 << SLOT_BITS) - 1), c >> SLOT_BITS))
        per.append(_count(waves, nrec))
    return {"path": "march", "N": N, "t": t, "ranks": ranks, "ring_records_per_slot": nrec}, per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", nargs="+", default=["fused:96:2:8:6", "fused:96:2:8:8", "fused:180:2:8:18",
                                                   "march:720:2:8"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    for spec in a.rows:
        f = spec.split(":")
        if f[0] == "fused":
            head, per = fused_row(*(int(x) for x in f[1:5]))
        else:
            head, per = march_row(*(int(x) for x in f[1:4]))
        mx = max(per, key=lambda d: d["records"])
        row = dict(head, max_rank={**mx, "ring_bytes": mx["records"] * mx["nw"] * 8, "payload_bytes": mx["records"] * 32,
                                   "tx_per_instr_aos": mx["tx_aos"] / max(1, mx["store_instr"]),
                                   "tx_per_instr_soa": mx["tx_soa"] / max(1, mx["store_instr"])},
                   total_records=sum(d["records"] for d in per))
        print(json.dumps(row), flush=True)
        if a.out:
            with open(a.out, "a") as fo:
                fo.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
