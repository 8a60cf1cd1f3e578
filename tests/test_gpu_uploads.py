"""The per-call upload ring under the node's threading contract, on the GPU.

A storage node serves decodes and recovery-symbol requests from many worker threads at once
(recovery_symbol_service.rs:251-267, node.rs:2615-2633), with plans, verifiers and caller
streams created and torn down between calls.  The engine moves each call's small uploads
(position offsets, multiplier logs, verifier targets) through a ring of 64 pinned slots; a slot
is reused once the copy kernel that read it has stored its generation in a completion word
(rs2_engine.cpp UploadSlots).  Round 5 guarded the slots with HIP events and fell back to a
device-wide synchronize when the event's stream had been destroyed; this test drives that case
(slots wrapping onto copies queued on streams, plans and verifiers destroyed since) and checks
that every decode and recovery symbol stays correct and that no device-wide synchronize is
taken (rs2_device_memory_stats slot 5 unchanged) while the ring wraps several times.
"""
import ctypes
import threading

import numpy as np
import pytest

import rs2_oracle as O

pytestmark = pytest.mark.gpu


def _hip():
    return ctypes.CDLL("libamdhip64.so")


def test_upload_ring_under_thread_and_stream_churn(gpu):
    import torch
    dev = torch.device("cuda", 0)
    n, length = 40, 123_457
    kp = O.source_symbols_for_n_shards(n)[0]
    blob = np.random.default_rng(11).integers(0, 256, length, dtype=np.uint8)
    b = torch.from_numpy(blob).to(dev)
    hip = _hip()
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]

    def encode(plan):
        info = plan.info
        prim = torch.zeros(n * info.primary_sliver_len + 256, dtype=torch.uint8, device=dev)
        sec = torch.zeros(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
        meta = torch.zeros(n * 64 + 32, dtype=torch.uint8, device=dev)
        plan.encode_async(b.data_ptr(), prim.data_ptr(), sec.data_ptr(), meta.data_ptr(),
                          meta[n * 64:].data_ptr())
        plan.sync()
        return prim, info

    from walrus_amd.encoding import device_memory_stats, upload_stats
    stats0 = device_memory_stats()
    up0 = upload_stats()
    errors = []
    iters = 72  # > 64 uploads per thread from the decodes alone (several uploads per decode)

    def worker(tid):
        try:
            rng = np.random.default_rng(100 + tid)
            plan = prim = info = None
            out = torch.zeros(length, dtype=torch.uint8, device=dev)
            for it in range(iters):
                if it % 9 == 0:  # a new plan; the old one (and its streams) destroyed
                    plan = None
                    plan = gpu.DevicePlan(n, length)
                    prim, info = encode(plan)
                pl = info.primary_sliver_len
                sel = [int(i) for i in rng.permutation(n)[:kp]]
                st = ctypes.c_void_p()
                assert hip.hipStreamCreate(ctypes.byref(st)) == 0
                out.zero_()
                torch.cuda.synchronize()
                plan.decode_async("primary", sel, prim.data_ptr(), [i * pl for i in sel],
                                  out.data_ptr(), st.value)
                assert hip.hipStreamSynchronize(st) == 0
                if not torch.equal(out, b):
                    errors.append(f"thread {tid} decode {it}: wrong blob")
                if it % 4 == 0:
                    # a fresh verifier per request batch: its target upload goes through the
                    # ring on the caller stream (odd iterations) or its own (even), then the
                    # verifier and its stream are destroyed
                    s = info.symbol_size
                    ver = gpu.SliverVerifier(n, s, "primary")
                    tg = [int(t) for t in rng.integers(0, n, 3)]
                    sym = torch.zeros(3 * s, dtype=torch.uint8, device=dev)
                    prf = torch.zeros(3 * 6 * 32, dtype=torch.uint8, device=dev)
                    own = (it // 4) % 2 == 0
                    ver.recovery_symbols_async(3, prim.data_ptr(), tg, sym.data_ptr(),
                                               prf.data_ptr(), 0, None if own else st.value)
                    if own:
                        del ver  # rs2_verifier_destroy waits for its stream, then destroys it
                    else:
                        assert hip.hipStreamSynchronize(st) == 0
                        del ver
                    torch.cuda.synchronize()
                    got = sym.cpu().numpy()
                    for r, t in enumerate(tg):
                        # primary sliver r's symbol t of its secondary-code expansion: for
                        # t < K_s that is the sliver's own symbol t
                        if t < info.n_secondary:
                            want = prim[r * pl + t * s:r * pl + (t + 1) * s].cpu().numpy()
                            if not np.array_equal(got[r * s:(r + 1) * s], want):
                                errors.append(f"thread {tid} request {it}: recovery symbol")
                assert hip.hipStreamDestroy(st) == 0
        except Exception as e:  # surfaced in the main thread
            errors.append(f"thread {tid}: {type(e).__name__}: {e}")

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in threads), "upload ring worker hung"
    assert not errors, errors[:5]
    up1 = upload_stats()
    # the ring wrapped several times over (64 slots)
    assert up1["uploads"] - up0["uploads"] > 4 * 64, (up0, up1)
    # and no device-wide synchronize was taken for it (nor by anything else in the test)
    assert device_memory_stats()["syncs"] == stats0["syncs"]
