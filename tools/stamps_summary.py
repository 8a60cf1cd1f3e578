"""Summarise in-kernel phase stamps (RS2_STAMP_FILE written by a -DRS2_STAMPS=1 library).

Each record: int32 {mode, C, tiles, n_z, kStamps, waves} then tiles*n_z*waves*kStamps uint64
s_memtime values (lane 0 of every wave of each workgroup, 0 = unused slot).  For every launch:
workgroup count, mean workgroup duration (first wave's first stamp to last wave's last stamp), and
per phase (delta to the previous stamp of the same wave): the mean over waves, wave 0's value,
the slowest wave's value, and the skew of the waves' arrival at the phase's end stamp.

usage: python tools/stamps_summary.py STAMP_FILE
"""
import struct
import sys

import numpy as np

MODES = {0: "rows", 1: "cols", 2: "decode", 3: "cols_pipe", 4: "rows_pipe"}


def records(path):
    raw = open(path, "rb").read()
    off = 0
    while off < len(raw):
        mode, C, tiles, n_z, k, nw = struct.unpack_from("6i", raw, off)
        off += 24
        n = tiles * n_z * nw * k
        st = np.frombuffer(raw, dtype=np.uint64, count=n, offset=off).reshape(tiles * n_z, nw, k)
        off += 8 * n
        yield mode, C, tiles, n_z, nw, st


def main(path):
    for mode, C, tiles, n_z, nw, st in records(path):
        used = (st != 0).any(axis=(0, 1))
        k = int(np.max(np.nonzero(used)[0])) + 1 if used.any() else 0
        if k < 2:
            continue
        st = st[:, :, :k].astype(np.int64)
        ok = (st != 0).all(axis=(1, 2))  # workgroups whose every wave wrote every stamp
        st = st[ok]
        if len(st) == 0:
            continue
        wg = st[:, :, -1].max(axis=1) - st[:, :, 0].min(axis=1)
        d = np.diff(st, axis=2)  # (wg, wave, phase)
        print(f"== {MODES.get(mode, mode)} C={C} workgroups={len(st)} (tiles {tiles} x z {n_z}, "
              f"{nw} waves) mean WG={wg.mean():.0f} ticks")
        print("   phase   mean-wave   wave0  slowest   end-skew   (ticks; % of WG on the mean)")
        for i in range(d.shape[2]):
            mean_w = d[:, :, i].mean()
            w0 = d[:, 0, i].mean()
            slow = d[:, :, i].max(axis=1).mean()
            skew = (st[:, :, i + 1].max(axis=1) - st[:, :, i + 1].min(axis=1)).mean()
            print(f"   {i + 1:5d} {mean_w:10.0f} {w0:8.0f} {slow:8.0f} {skew:10.0f}   "
                  f"{100 * mean_w / wg.mean():5.1f} %")


if __name__ == "__main__":
    main(sys.argv[1])
