"""Recovery symbols with Merkle proofs, sliver recovery and inconsistency proofs on the GPU.

Mirrors the reference's own tests:
  symbols.rs:784-828   test_recovery_symbol_proof (GeneralRecoverySymbol, both axes)
  slivers.rs:832-861   test_recovery_symbol_proof (2- and 4-byte symbols vs the sliver's tree)
  inconsistency.rs:209-286  valid / wrong target / not inconsistent / too few symbols
  merkle.rs:353-465    proofs for every leaf, against the tree root
and checks every symbol and proof byte against the CPU oracle's MerkleTree::get_proof
restatement (oracle/rs2_oracle.py merkle_proof, test infrastructure only).  The reference's
tests build configs with non-default (K_p, K_s) via EncodingConfig::new_for_test; the engine
derives them from n_shards as production does, so the same properties are checked at the
derived parameters.
"""
import numpy as np
import pytest

import rs2_oracle as O

pytestmark = pytest.mark.gpu


def _encode(gpu, n, length, seed):
    blob = np.random.default_rng(seed).integers(0, 256, length, dtype=np.uint8).tobytes()
    cfg = gpu.ReedSolomonEncodingConfig(n)
    pairs, meta = cfg.encode_with_metadata(blob)
    return cfg, pairs, meta, blob


def _params(cfg, length):
    kp, ks = cfg.n_primary_source_symbols, cfg.n_secondary_source_symbols
    return O.Rs2Params(cfg.n_shards, kp, ks, cfg.symbol_size_for_blob(length), length)


@pytest.mark.parametrize("n,length", [(4, 50), (7, 257), (10, 1000), (100, 40_000),
                                      (1000, 3_000_000)])
def test_recovery_symbols_match_oracle(gpu, n, length):
    cfg, pairs, meta, blob = _encode(gpu, n, length, n + length)
    p = _params(cfg, length)
    rng = np.random.default_rng(n)
    sources = [pairs[int(i)].primary for i in rng.permutation(n)[:3]] + \
              [pairs[int(i)].secondary for i in rng.permutation(n)[:3]]
    targets = [int(t) for t in rng.integers(0, n, len(sources))]
    if n <= 10:  # every (source, target) pair
        sources = [sl for sl in sources for _ in range(n)]
        targets = list(range(n)) * 6
    syms = gpu.recovery_symbols_for_requests(cfg, sources, targets)
    for sl, tp, rs in zip(sources, targets, syms):
        orth = gpu.SECONDARY if sl.axis == gpu.PRIMARY else gpu.PRIMARY
        t_sliver = tp if orth == gpu.PRIMARY else n - 1 - tp
        exp = O.recovery_symbols(np.frombuffer(sl.symbols.data, np.uint8), sl.axis, p)
        leaves = [exp[i].tobytes() for i in range(n)]
        assert rs.axis == orth and rs.index == sl.index
        assert rs.data == leaves[t_sliver]
        assert rs.proof.path == O.merkle_proof(leaves, t_sliver)
        # verifies against the metadata at its target, and not at another one
        rs.verify(n, p.symbol_size, meta.metadata, t_sliver)
        if n > 1:
            with pytest.raises(gpu.recovery.SymbolVerificationError):
                rs.verify(n, p.symbol_size, meta.metadata, (t_sliver + 1) % n)
        # and it is the decoding symbol the reference derives without a proof
        assert sl.decoding_symbol_for_sliver(tp, cfg).data == rs.data


def test_general_recovery_symbol_both_axes(gpu):
    """symbols.rs:784-828 (n = 7, blob of 257 bytes, source = secondary sliver of pair 0)."""
    n = 7
    cfg, pairs, meta, _ = _encode(gpu, n, 257, 1)
    sliver = pairs[0].secondary
    source_index = n - 1  # SliverPairIndex(0).to_sliver_index::<Secondary>
    for index in range(n):
        sym = gpu.recovery_symbol_for_sliver(sliver, index, cfg)
        g = gpu.GeneralRecoverySymbol(sym, index)
        g.verify(meta.metadata, cfg, index, gpu.PRIMARY)
        g.verify(meta.metadata, cfg, source_index, gpu.SECONDARY)
        other = next(t for t in range(n) if t not in (index, source_index))
        with pytest.raises(gpu.recovery.SymbolVerificationError) as e:
            g.verify(meta.metadata, cfg, other, gpu.PRIMARY)
        assert e.value.kind == "SymbolNotUsable"


@pytest.mark.parametrize("symbol_size", [2, 4])
def test_recovery_symbol_proof_vs_tree_root(gpu, symbol_size):
    """slivers.rs:832-861: a bare secondary sliver; every pair index's recovery symbol verifies
    against the Merkle root of the sliver's expansion (n = 7: K_p = 3 symbols)."""
    n = 7
    cfg = gpu.ReedSolomonEncodingConfig(n)
    kp = cfg.n_primary_source_symbols
    data = bytes(range(1, kp * symbol_size + 1))
    sliver = gpu.SliverData(gpu.Symbols(data, symbol_size), 0, gpu.SECONDARY)
    root = sliver.get_merkle_root(cfg)
    exp = sliver.recovery_symbols(cfg)
    assert root == O.merkle_root(exp.to_symbols())
    for index in range(n):
        sym = gpu.recovery_symbol_for_sliver(sliver, index, cfg)
        sym.verify_proof(root, n, index)


def test_merkle_proof_roots_every_leaf(gpu):
    """merkle.rs:353-465: a proof for every leaf of trees of 1..40 leaves recomputes the root;
    wrong index / leaf / over-long path are rejected."""
    from walrus_amd.recovery import MerkleProof, MerkleProofError, compute_roots
    rng = np.random.default_rng(3)
    proofs, leaves, idxs, roots = [], [], [], []
    for m in list(range(1, 41)) + [255, 256, 257, 1000]:
        data = [rng.integers(0, 256, 6, dtype=np.uint8).tobytes() for _ in range(m)]
        root = O.merkle_root(data)
        for i in (range(m) if m <= 40 else rng.integers(0, m, 8)):
            proofs.append(MerkleProof(O.merkle_proof(data, int(i))))
            leaves.append(data[int(i)])
            idxs.append(int(i))
            roots.append(root)
    got = compute_roots(proofs, leaves, idxs)
    assert got == roots
    p = proofs[-1]
    p.verify_proof(roots[-1], 1000, leaves[-1], idxs[-1])
    with pytest.raises(MerkleProofError):
        p.verify_proof(roots[-1], 1000, leaves[-1], idxs[-1] ^ 1)
    with pytest.raises(MerkleProofError):
        p.verify_proof(roots[-1], 1000, b"\0" * 6, idxs[-1])
    with pytest.raises(MerkleProofError) as e:
        MerkleProof(p.path + [b"\0" * 32]).verify_proof(roots[-1], 1000, leaves[-1], idxs[-1])
    assert e.value.kind == "PathLengthTooLarge"
    with pytest.raises(MerkleProofError) as e:
        MerkleProof([]).compute_root(b"ab", 1)
    assert e.value.kind == "LeafIndexOutOfBounds"


def _inconsistency_setup(gpu):
    """test_utils.rs:325-352: blob of 314 bytes, target primary sliver 0, a random subset of
    n_symbols_for_recovery secondary-sliver recovery symbols (pairs 1..n)."""
    n = 10
    cfg, pairs, meta, _ = _encode(gpu, n, 314, 42)
    need = cfg.n_symbols_for_recovery(gpu.PRIMARY)
    chosen = [int(i) for i in np.random.default_rng(42).permutation(np.arange(1, n))[:need]]
    syms = gpu.recovery_symbols_for_requests(cfg, [pairs[i].secondary for i in chosen],
                                             [0] * need)
    return cfg, pairs, meta, syms


def test_inconsistency_proofs(gpu):
    R = gpu.recovery
    cfg, pairs, meta, syms = _inconsistency_setup(gpu)
    md = meta.metadata
    bad = gpu.BlobMetadata([(b"\0" * 32, h[1]) if i == 0 else h
                            for i, h in enumerate(md.hashes)], md.unencoded_length)
    # valid_inconsistency_proof
    gpu.InconsistencyProof(gpu.PRIMARY, 0, syms).verify(bad, cfg)
    # invalid_inconsistency_proof_when_just_changing_the_target_index
    with pytest.raises(R.InconsistencyVerificationError) as e:
        gpu.InconsistencyProof(gpu.PRIMARY, 1, syms).verify(md, cfg)
    assert e.value.kind == "InvalidRecoverySymbols"
    # invalid_inconsistency_proof_because_sliver_not_inconsistent
    with pytest.raises(R.InconsistencyVerificationError) as e:
        gpu.InconsistencyProof(gpu.PRIMARY, 0, syms).verify(md, cfg)
    assert e.value.kind == "SliverNotInconsistent"
    # invalid_inconsistency_proof_because_of_insufficient_recovery_symbols
    with pytest.raises(R.InconsistencyVerificationError) as e:
        gpu.InconsistencyProof(gpu.PRIMARY, 0, syms[:-1]).verify(md, cfg)
    assert e.value.kind == "IncorrectSymbolCount"
    assert e.value.detail == (len(syms), len(syms) - 1)


def test_recover_sliver_or_inconsistency_proof(gpu):
    """slivers.rs:341-379: a consistent blob gives back the sliver, a contradicting metadata
    hash gives an InconsistencyProof that verifies; both sliver axes."""
    cfg, pairs, meta, syms = _inconsistency_setup(gpu)
    md = meta.metadata
    got = gpu.recover_sliver_or_generate_inconsistency_proof(syms + syms[:2], 0, md, cfg,
                                                             gpu.PRIMARY)
    assert isinstance(got, gpu.SliverData) and got.symbols.data == pairs[0].primary.symbols.data
    bad = gpu.BlobMetadata([(b"\0" * 32, h[1]) if i == 0 else h
                            for i, h in enumerate(md.hashes)], md.unencoded_length)
    proof = gpu.recover_sliver_or_generate_inconsistency_proof(syms, 0, bad, cfg, gpu.PRIMARY)
    assert isinstance(proof, gpu.InconsistencyProof)
    proof.verify(bad, cfg)
    # secondary target: sliver n-1 (pair 0) from primary slivers' recovery symbols
    n = cfg.n_shards
    need = cfg.n_symbols_for_recovery(gpu.SECONDARY)
    src = [pairs[i].primary for i in range(1, 1 + need)]
    ssyms = gpu.recovery_symbols_for_requests(cfg, src, [0] * need)
    got = gpu.recover_sliver_or_generate_inconsistency_proof(ssyms, n - 1, md, cfg,
                                                             gpu.SECONDARY)
    assert got.symbols.data == pairs[0].secondary.symbols.data
    # try_recover_sliver_from_decoding_symbols (no proofs), and too few symbols
    dsyms = [s.into_decoding_symbol() for s in ssyms]
    assert gpu.try_recover_sliver_from_decoding_symbols(
        dsyms, n - 1, md, cfg, gpu.SECONDARY).symbols.data == pairs[0].secondary.symbols.data
    with pytest.raises(gpu.recovery.SliverRecoveryError):
        gpu.try_recover_sliver_from_decoding_symbols(dsyms[:-1], n - 1, md, cfg, gpu.SECONDARY)


def test_recovery_symbols_device_nodes(gpu):
    """rs2_verifier_recovery_symbols_device_async: the full trees it returns are the
    reference's MerkleTree::nodes arrays (what the node's service caches)."""
    import ctypes
    import torch
    from walrus_amd import _lib
    from walrus_amd.encoding import _ok
    n = 100
    cfg, pairs, meta, blob = _encode(gpu, n, 20_000, 9)
    p = _params(cfg, len(blob))
    s = p.symbol_size
    v = gpu.SliverVerifier(n, s, gpu.PRIMARY)
    src = [pairs[i].primary for i in (3, 50, 99)]
    dev = torch.device("cuda", 0)
    d_sl = torch.tensor(np.frombuffer(b"".join(x.symbols.data for x in src), np.uint8),
                        device=dev)
    L = gpu.recovery.path_length(n)
    nn = ctypes.c_uint64()
    _ok(_lib.lib().rs2_merkle_tree_shape(n, None, ctypes.byref(nn)))
    d_sym = torch.zeros(3 * s, dtype=torch.uint8, device=dev)
    d_prf = torch.zeros(3 * L * 32, dtype=torch.uint8, device=dev)
    d_nodes = torch.zeros(3 * nn.value * 32, dtype=torch.uint8, device=dev)
    tg = (ctypes.c_uint16 * 3)(0, 57, 99)
    _ok(_lib.lib().rs2_verifier_recovery_symbols_device_async(
        v.handle, 3, d_sl.data_ptr(), tg, d_sym.data_ptr(), d_prf.data_ptr(), d_nodes.data_ptr(),
        None))
    torch.cuda.synchronize()
    nodes = d_nodes.cpu().numpy().tobytes()
    for k, x in enumerate(src):
        exp = O.recovery_symbols(np.frombuffer(x.symbols.data, np.uint8), gpu.PRIMARY, p)
        want = b"".join(O.merkle_nodes([exp[i].tobytes() for i in range(n)]))
        assert nodes[k * nn.value * 32:(k + 1) * nn.value * 32] == want
        assert d_sym[k * s:(k + 1) * s].cpu().numpy().tobytes() == exp[tg[k]].tobytes()


def test_verifier_destroy_waits_for_caller_stream(gpu):
    """rs2_verifier_destroy with roots still queued on a caller's stream: the verifier's arena
    ranges must not be handed to the next plan before that work has run.  The
    caller stream is held back by a spin kernel, the verifier is dropped, a new plan encodes on
    another stream over the freed ranges, and the queued roots must still be the right ones."""
    import gc
    import torch
    n = 1000
    cfg, pairs, meta, blob = _encode(gpu, n, 2_000_000, 11)
    s = cfg.symbol_size_for_blob(len(blob))
    dev = torch.device("cuda", 0)
    rows = list(range(0, n, 7))
    d_sl = torch.tensor(np.frombuffer(b"".join(pairs[i].primary.symbols.data for i in rows),
                                      np.uint8), device=dev)
    d_roots = torch.zeros(len(rows) * 32, dtype=torch.uint8, device=dev)
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        torch.cuda._sleep(200_000_000)  # ~0.1 s of queued work ahead of the roots
    v = gpu.SliverVerifier(n, s, gpu.PRIMARY)
    v.roots_async(len(rows), d_sl.data_ptr(), d_roots.data_ptr(), side.cuda_stream)
    del v
    gc.collect()
    other = np.random.default_rng(12).integers(0, 256, 3_000_000, dtype=np.uint8).tobytes()
    plan = gpu.DevicePlan(n, len(other))
    info = plan.info
    b = torch.tensor(np.frombuffer(other, np.uint8), device=dev)
    prim = torch.empty(n * info.primary_sliver_len + 256, dtype=torch.uint8, device=dev)
    sec = torch.empty(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
    hashes = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    bid = torch.empty(32, dtype=torch.uint8, device=dev)
    plan.encode_async(b.data_ptr(), prim.data_ptr(), sec.data_ptr(), hashes.data_ptr(),
                      bid.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    got = d_roots.cpu().numpy().tobytes()
    for k, i in enumerate(rows):
        assert got[32 * k:32 * k + 32] == meta.metadata.hashes[i][0], i


@pytest.fixture(scope="module")
def cpu_port():
    import ctypes
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_fullsize import load_cpu
    lib = load_cpu()
    P = ctypes.c_void_p
    lib.rs2cpu_recovery_symbol.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, P,
                                           ctypes.c_uint32, P, P]
    lib.rs2cpu_sliver_root.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, P, P]
    return lib


@pytest.mark.parametrize("n", [4097, 6000, 24600, 49155])
def test_recovery_symbols_wide_trees(gpu, cpu_port, n):
    """Recovery symbols and proofs for n_shards above 4,096 (full node arrays built one level per
    launch through HBM, rs2_hash.hip merkle_nodes_level_kernel) against the C restatement's
    rs2cpu_recovery_symbol (MerkleTree::get_proof, merkle.rs:281-309), on both axes, for
    arbitrary sliver bytes (the recovery symbol is defined for any sliver)."""
    import ctypes
    from walrus_amd import _lib
    from walrus_amd.encoding import _ok
    cfg = gpu.ReedSolomonEncodingConfig(n)
    kp, ks = cfg.n_primary_source_symbols, cfg.n_secondary_source_symbols
    s = 4
    L = gpu.recovery.path_length(n)
    rng = np.random.default_rng(n)
    for axis, k in ((0, ks), (1, kp)):
        slivers = [rng.integers(0, 256, k * s, dtype=np.uint8) for _ in range(3)]
        targets = [0, n - 1, int(rng.integers(0, n))]
        ptrs = (ctypes.c_void_p * 3)(*[a.ctypes.data for a in slivers])
        lens = (ctypes.c_uint64 * 3)(*[k * s] * 3)
        ta = (ctypes.c_uint16 * 3)(*targets)
        syms = np.zeros(3 * s, np.uint8)
        proofs = np.zeros(3 * L * 32, np.uint8)
        _ok(_lib.lib().rs2_recovery_symbols(n, s, axis, 3, ptrs, lens, ta, syms.ctypes.data,
                                            proofs.ctypes.data))
        sym = np.zeros(s, np.uint8)
        prf = np.zeros(L * 32, np.uint8)
        for i, (sl, t) in enumerate(zip(slivers, targets)):
            assert cpu_port.rs2cpu_recovery_symbol(n, s, axis, sl.ctypes.data, t, sym.ctypes.data,
                                                   prf.ctypes.data) == L
            assert syms[i * s:(i + 1) * s].tobytes() == sym.tobytes(), (axis, i)
            assert proofs[i * L * 32:(i + 1) * L * 32].tobytes() == prf.tobytes(), (axis, i)


def test_recovery_symbols_device_nodes_wide(gpu, cpu_port):
    """The full node array of a 6,000-leaf tree (MerkleTree::nodes order: levels padded to even
    with the zero node, root last): every inner node is inner(left, right) of the level below,
    the root is the C restatement's sliver root, and the proof read from it matches."""
    import ctypes
    import hashlib
    import torch
    from walrus_amd import _lib
    from walrus_amd.encoding import _ok
    n, s = 6000, 2
    cfg = gpu.ReedSolomonEncodingConfig(n)
    k = cfg.n_secondary_source_symbols
    sl = np.random.default_rng(1).integers(0, 256, k * s, dtype=np.uint8)
    v = gpu.SliverVerifier(n, s, gpu.PRIMARY)
    dev = torch.device("cuda", 0)
    d_sl = torch.from_numpy(sl.copy()).to(dev)
    L = gpu.recovery.path_length(n)
    nn = ctypes.c_uint64()
    _ok(_lib.lib().rs2_merkle_tree_shape(n, None, ctypes.byref(nn)))
    d_sym = torch.zeros(s, dtype=torch.uint8, device=dev)
    d_prf = torch.zeros(L * 32, dtype=torch.uint8, device=dev)
    d_nodes = torch.full((nn.value * 32,), 0xAB, dtype=torch.uint8, device=dev)
    tg = (ctypes.c_uint16 * 1)(4321)
    _ok(_lib.lib().rs2_verifier_recovery_symbols_device_async(
        v.handle, 1, d_sl.data_ptr(), tg, d_sym.data_ptr(), d_prf.data_ptr(), d_nodes.data_ptr(),
        None))
    torch.cuda.synchronize()
    nodes = d_nodes.cpu().numpy().reshape(-1, 32)
    cnt, base = n, 0
    while cnt > 1:
        if cnt & 1:
            assert not nodes[base + cnt].any()
            cnt += 1
        for j in range(cnt // 2):
            h = hashlib.blake2b(b"\x01" + nodes[base + 2 * j].tobytes() +
                                nodes[base + 2 * j + 1].tobytes(), digest_size=32).digest()
            assert nodes[base + cnt + j].tobytes() == h, (base, j)
        base += cnt
        cnt //= 2
    assert base + 1 == nn.value
    root = np.zeros(32, np.uint8)
    cpu_port.rs2cpu_sliver_root(n, s, 0, sl.ctypes.data, root.ctypes.data)
    assert nodes[-1].tobytes() == root.tobytes()
    sym = np.zeros(s, np.uint8)
    prf = np.zeros(L * 32, np.uint8)
    cpu_port.rs2cpu_recovery_symbol(n, s, 0, sl.ctypes.data, 4321, sym.ctypes.data,
                                    prf.ctypes.data)
    assert d_prf.cpu().numpy().tobytes() == prf.tobytes()
    assert d_sym.cpu().numpy().tobytes() == sym.tobytes()


@pytest.mark.parametrize("n", [4500, 24600])
def test_recover_sliver_wide(gpu, n):
    """recover_sliver_or_generate_inconsistency_proof above 4,096 shards (recovery symbols with
    proofs from wide trees, their verification, the 1D decode of the target sliver at 8192 /
    65536-point transforms and its root check): primary sliver 5 from K_s secondary slivers'
    symbols and secondary sliver n-1 from K_p primary slivers' symbols, against the encode."""
    cfg, pairs, meta, _ = _encode(gpu, n, 1 << 20, n)
    md = meta.metadata
    rng = np.random.default_rng(n)
    need = cfg.n_symbols_for_recovery(gpu.PRIMARY)
    src = [pairs[int(i)].secondary for i in rng.permutation(n)[:need]]
    syms = gpu.recovery_symbols_for_requests(cfg, src, [5] * need)
    got = gpu.recover_sliver_or_generate_inconsistency_proof(syms, 5, md, cfg, gpu.PRIMARY)
    assert isinstance(got, gpu.SliverData) and got.symbols.data == pairs[5].primary.symbols.data
    need = cfg.n_symbols_for_recovery(gpu.SECONDARY)
    src = [pairs[int(i)].primary for i in rng.permutation(n)[:need]]
    syms = gpu.recovery_symbols_for_requests(cfg, src, [0] * need)
    got = gpu.recover_sliver_or_generate_inconsistency_proof(syms, n - 1, md, cfg, gpu.SECONDARY)
    assert got.symbols.data == pairs[0].secondary.symbols.data
