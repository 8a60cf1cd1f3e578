"""The engine's A/B kernel variants give the same bytes as the default kernels.

The defaults run the decode block pair (rs2_codec.hip load_ifft, CodecJob::pair_p) and the
tile-pipelined encode kernels (pipe_body); RS2_PAIR=0 / RS2_PIPE=0 select the single-block decode
pass and the one-tile encode kernels, RS2_PIPE_DYN=1 the pipelined kernels' dynamic tile order,
RS2_DEC_PERSIST=1 the persistent decode kernel, RS2_LEAF_WIN=2 two message blocks per leaf-hash
window, RS2_BLOCK_MAX=256 transform blocks of 256 positions (twice the block mixing), and the
stage-fusion knobs RS2_FUSE_BLOB=0 / RS2_TAIL_AUX=1 / RS2_SPLIT_LEAF=0 / RS2_DEC_NOFUSE=1 /
RS2_SMALL_LEAF=0 their unfused forms.  The knobs are read once per process, so the variant runs
in a child process and reports digests of its slivers, metadata and decodes; the parent compares
them with its own (default) run and with the CPU oracle's encode at the small shape.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import rs2_oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (n_shards, blob bytes): n = 1000 pairs decode blocks 0 and 2 and pipelines both encode codes;
# the others cover smaller transform blocks (C = 128 / 64) and the shapes that do not pipeline
# (n = 1000 at 3 MB has s = 14: the one-block leaf kernel; 70 MB, s = 316, and n = 40, s = 266,
# run the LDS-window leaf kernel; 70 MB is above the 64 MiB where the encode splits its leaf
# hashing and runs the tail rows on their own stream)
SHAPES = [(1000, 3_000_000), (1000, 70_000_000), (300, 700_000), (100, 123_457), (40, 100_000)]


def digests(shapes):
    import walrus_amd as W
    out = {}
    for n, blob_len in shapes:
        rng = np.random.default_rng(n + blob_len)
        blob = rng.integers(0, 256, blob_len, dtype=np.uint8).tobytes()
        cfg = W.ReedSolomonEncodingConfig(n)
        pairs, meta = cfg.encode_with_metadata(blob)
        h = hashlib.sha256()
        for p in pairs:
            h.update(p.primary.symbols.data)
            h.update(p.secondary.symbols.data)
        order = rng.permutation(n)
        dec = cfg.decode(blob_len, [pairs[i].primary for i in order])
        worst = cfg.decode(blob_len, [pairs[i].primary for i in range(n - 1, -1, -1)])
        sec = cfg.decode(blob_len, [pairs[n - 1 - i].secondary for i in order])
        out[f"{n}/{blob_len}"] = {
            "slivers": h.hexdigest(), "blob_id": bytes(meta.blob_id).hex(),
            "decodes_ok": dec == blob and worst == blob and sec == blob}
    return out


def test_variants_match_default(gpu):
    base = digests(SHAPES)
    assert all(v["decodes_ok"] for v in base.values()), base
    # the small shape against the oracle too (the defaults are what every other test checks)
    n, blob_len = SHAPES[-1]
    rng = np.random.default_rng(n + blob_len)
    blob = rng.integers(0, 256, blob_len, dtype=np.uint8).tobytes()
    assert base[f"{n}/{blob_len}"]["blob_id"] == O.encode_with_metadata(blob, n).blob_id.hex()
    code = ("import json, sys; sys.path[:0] = %r; "
            "import test_gpu_variants as T; print(json.dumps(T.digests(T.SHAPES)))"
            % ([ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")],))
    for env in ({"RS2_PAIR": "0", "RS2_PIPE": "0"}, {"RS2_PIPE": "2"}, {"RS2_DEC_PERSIST": "1"},
                {"RS2_PIPE_DYN": "1"}, {"RS2_LEAF_WIN": "2"}, {"RS2_BLOCK_MAX": "256"},
                {"RS2_FUSE_BLOB": "0", "RS2_TAIL_AUX": "1", "RS2_SPLIT_LEAF": "0",
                 "RS2_DEC_NOFUSE": "1", "RS2_SMALL_LEAF": "0"}):
        r = subprocess.run([sys.executable, "-c", code], env={**os.environ, **env},
                           capture_output=True, text=True, timeout=240, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-2000:]
        got = json.loads(r.stdout.strip().splitlines()[-1])
        assert got == base, (env, got, base)
