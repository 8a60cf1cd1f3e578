"""CPU checker with the `ops` interface of walrus_amd.partition.DeviceOps -- TEST ONLY.

Backed by the numpy oracle (oracle/rs2_oracle.py), it lets the partitioned (multi-rank) encode
and decode run on CPU torch tensors over gloo, so the partitioning and the exchanges are
tested without a GPU.  Never used by the product path (DeviceOps is the HIP engine).
"""
import hashlib

import numpy as np
import rs2_oracle as O


def _np(t):
    """Flat byte view of a contiguous CPU tensor (the device ops take byte offsets)."""
    return t.numpy().reshape(-1)


class CpuOps:
    def offsets(self, key, build, device):
        a = np.ascontiguousarray(build(), dtype=np.int64)
        return a, int(np.gcd.reduce(a)) if a.size else 0

    def copy_segments(self, src, dst, src_a, dst_a, count_b, ssb, dsb, seg_len):
        a, d = _np(src), _np(dst)
        for so, do in zip(src_a[0], dst_a[0]):
            for b in range(count_b):
                x, y = int(so) + b * ssb, int(do) + b * dsb
                d[y:y + seg_len] = a[x:x + seg_len]

    def encode_lines(self, k, n, s, lines, src, src_off, src_ss, src_ls, dst, dst_off, dst_ss,
                     dst_ls):
        a, d = _np(src), _np(dst)
        for line in range(lines):
            base = src_off + line * src_ls
            data = np.stack([a[base + i * src_ss: base + i * src_ss + s] for i in range(k)])
            rep = O.rs_encode_symbols(data, n - k)
            ob = dst_off + line * dst_ls
            for j in range(n - k):
                d[ob + j * dst_ss: ob + j * dst_ss + s] = rep[j]

    def decode_lines(self, k, n, s, lines, idx, base, sym_off, line_stride, out, out_ss, out_ls,
                     out_limit):
        a, d = _np(base), _np(out)
        for line in range(lines):
            syms = [(int(q), a[o + line * line_stride: o + line * line_stride + s])
                    for q, o in zip(idx, sym_off)]
            dec = O.rs_decode_symbols(k, n, s, syms)
            for i in range(k):
                o = line * out_ls + i * out_ss
                m = max(0, min(s, out_limit - o))
                d[o:o + m] = dec[i][:m]

    def leaf_hashes(self, symbols, count, s, out):
        a, d = _np(symbols), _np(out)
        for i in range(count):
            d[32 * i:32 * i + 32] = np.frombuffer(
                hashlib.blake2b(b"\x00" + a[i * s:(i + 1) * s].tobytes(), digest_size=32).digest(),
                dtype=np.uint8)

    def merkle_roots(self, leaves, n_trees, n_leaves, tree_stride, leaf_stride, out, root_stride):
        a, d = _np(leaves), _np(out)
        for t in range(n_trees):
            ls = [a[t * tree_stride + i * leaf_stride: t * tree_stride + i * leaf_stride + 32]
                  .tobytes() for i in range(n_leaves)]
            d[t * root_stride: t * root_stride + 32] = np.frombuffer(
                O.merkle_root_from_leaf_hashes(ls), dtype=np.uint8)

    def blob_id(self, hashes, n, blob_len, out):
        h = _np(hashes)[:n * 64].tobytes()
        pairs = [(h[64 * i:64 * i + 32], h[64 * i + 32:64 * i + 64]) for i in range(n)]
        _np(out)[:32] = np.frombuffer(O.blob_id(pairs, blob_len), dtype=np.uint8)
