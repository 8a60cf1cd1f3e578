"""Summarise in-kernel phase stamps (RS2_STAMP_FILE written by a -DRS2_STAMPS=1 library).

Each record: int32 {mode, C, tiles, n_z, kStamps} then tiles*n_z*kStamps uint64 s_memtime values
(wave 0 of each workgroup, 0 = unused slot).  For every launch: workgroup count, span, mean
workgroup duration, and the mean time of each phase (delta to the previous stamp), in ticks and
as a share of the workgroup duration.

usage: python tools/stamps_summary.py STAMP_FILE [labels...]
"""
import struct
import sys

import numpy as np

MODES = {0: "rows", 1: "cols", 2: "decode"}
LOAD_LABELS = ["issue loads+DMA", "wait loads", "pre-mul", "in-wave IFFT", "transpose A->B",
               "cross-wave IFFT"]


def records(path):
    raw = open(path, "rb").read()
    off = 0
    while off < len(raw):
        mode, C, tiles, n_z, k = struct.unpack_from("5i", raw, off)
        off += 20
        n = tiles * n_z * k
        st = np.frombuffer(raw, dtype=np.uint64, count=n, offset=off).reshape(tiles * n_z, k)
        off += 8 * n
        yield mode, C, tiles, n_z, st


def main(path):
    for mode, C, tiles, n_z, st in records(path):
        used = (st != 0).sum(axis=0)
        k = int(np.max(np.nonzero(used)[0])) + 1 if used.any() else 0
        st = st[:, :k].astype(np.int64)
        rows = (st[:, :k] != 0).all(axis=1)
        st = st[rows]
        if len(st) == 0:
            continue
        d = np.diff(st, axis=1)
        wg = st[:, -1] - st[:, 0]
        span = st[:, -1].max() - st[:, 0].min()
        conc = wg.sum() / span
        print(f"== {MODES.get(mode, mode)} C={C} workgroups={len(st)} (tiles {tiles} x z {n_z}) "
              f"span={span} ticks, mean WG={wg.mean():.0f} ticks, mean concurrency={conc:.1f}")
        for i in range(d.shape[1]):
            print(f"   phase {i + 1:2d}: {d[:, i].mean():9.0f} ticks  {100 * d[:, i].mean() / wg.mean():5.1f} %"
                  f"   (p10 {np.percentile(d[:, i], 10):.0f}, p90 {np.percentile(d[:, i], 90):.0f})")


if __name__ == "__main__":
    main(sys.argv[1])
