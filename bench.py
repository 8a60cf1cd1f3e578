#!/usr/bin/env python3
"""Red Stuff encode+decode GiB/s (device-resident), 256 MiB blob, n_shards=1000, 1..8 MI355X.

One step = BlobEncoder::encode_with_metadata of a 256 MiB blob (primary + secondary slivers,
n^2 leaf hashes, 2n Merkle trees, BlobId) followed by BlobDecoder::decode of the blob from a
seeded random subset of K_p = 334 primary slivers (the reference's criterion harness,
crates/walrus-core/benches/blob_encoding.rs:35-122), all inputs and outputs resident in HBM.
Every step draws its own subset (--subsets fresh, the default): a client read sees a new sliver
subset per blob, so the decoder's per-erasure-pattern setup (basic_encoding.rs:387-429: the
locator FWHT, here also the block mixing, the table uploads and the multiplier-table kernel) is
paid every step; --subsets fixed reuses one subset, as the criterion harness does.
GiB/s counts unencoded blob bytes (criterion Throughput::Bytes, blob_encoding.rs:42,88).

Multi-GPU: one process per GPU (torchrun; `--gpus N` without a torchrun environment launches
it); every rank encodes+decodes its own blob (weak scaling, independent blobs, no collective on
the data path).  value = all ranks' blob bytes over the max-over-ranks wall time of the timed
steps.  Beside the metric, at every N: config C3 (128 independent 4 MiB blobs dealt over the
ranks, BlobIds all-gathered) and config C4 (one 4 GiB blob row/column-partitioned over the
ranks with RCCL all-to-alls / all-gather, every rank ending with its assembled sliver pairs;
decoded from K_p primary slivers scattered from rank 0 and gathered back), each timed
max-over-ranks.

Output: one JSON line on rank 0 (see the driver contract in the task statement).
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); measured float4 copy 6290
# vector issue ceiling (MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2 cycles on a
# SIMD; 256 CUs x 4 SIMDs; 2.4 GHz peak engine clock)
VALU_CYC, SIMDS, CLOCK_HZ = 2, 1024, 2.4e9
# LDS: one array per CU, 2 LDS cycles per conflict-free ds_read_b32 / ds_read_u16 wave-instruction
# (MI355X_MICROARCH.md §LDS); the codecs' table lookups are those
LDS_CYC, CUS = 2, 256
# Not every VALU instruction issues in 2 cycles on gfx950: tools/micro/valubench measured ~2.1
# for the VOP1/VOP2 integer forms, ~2.35 for VOP3 / v_bitop3 and ~4.1 for SDWA, DPP, left shifts,
# v_perm / v_alignbit, 64-bit ops and SGPR operands.  tools/isa_mix.py prices each kernel's
# VALU mix from the library's ISA (profiles/isa_mix.json); the issue fractions below use that
# mean cycles-per-instruction per kernel (valu_issue_frac), beside the flat 2-cycle figure
# (valu_issue_frac_2cyc) the earlier rounds reported.
STAGE_ISA = {
    "enc_rows_codec": "rs2_encode_mixed_pipe_kernel<512>",
    "enc_cols_sys_codec": "rs2_encode_shared_pipe_kernel<512>",
    "enc_cols_rep_codec": "rs2_encode_shared_pipe_kernel<512>",
    "enc_leaf_hash": "leaf_hash_kernel<1>",
    "enc_leaf_hash_a": "leaf_hash_kernel<1>",
    "enc_merkle_trees": "merkle_trees_kernel",
    "enc_merkle_root": "merkle_root_kernel",
    "enc_tail_rows": "tail_rows_kernel",
    "dec_setup": "build_mul_tables_kernel",
    "dec_codec": "rs2_decode_kernel<512>",
}


class _ClockSampler:
    """Diagnostic (RS2_BENCH_CLOCKS=1): the GPU's graphics clock and socket power, sampled every
    ~2 ms by a host thread through amdsmi (read-only queries), tagged with the bench phase.
    Round 5 read the solo decode 10 % above its isolated launch; the solo pass runs right after
    the timed region, and this shows the clock it runs at."""

    def __init__(self, local_rank: int):
        import threading
        import amdsmi
        self.smi = amdsmi
        amdsmi.amdsmi_init()
        hs = amdsmi.amdsmi_get_processor_handles()
        self.h = hs[min(local_rank, len(hs) - 1)]
        self.samples = []
        self.phase = "setup"
        self._stop = False
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        t0 = time.perf_counter()
        while not self._stop:
            try:
                clk = self.smi.amdsmi_get_clock_info(self.h, self.smi.AmdSmiClkType.SYS)["clk"]
            except Exception:
                clk = None
            other = {}
            for name in ("MEM", "DF", "SOC"):
                try:
                    other[name] = self.smi.amdsmi_get_clock_info(
                        self.h, getattr(self.smi.AmdSmiClkType, name))["clk"]
                except Exception:
                    other[name] = None
            try:
                m = self.smi.amdsmi_get_gpu_metrics_info(self.h)
                pw = m.get("current_socket_power") or m.get("average_socket_power")
            except Exception:
                pw = None
            self.samples.append((time.perf_counter() - t0, self.phase, clk, pw, other))
            time.sleep(0.002)

    def summary(self):
        self._stop = True
        self._t.join(timeout=1)
        out = {}
        for ph in dict.fromkeys(s[1] for s in self.samples):
            c = [s[2] for s in self.samples if s[1] == ph and isinstance(s[2], (int, float))]
            w = [s[3] for s in self.samples if s[1] == ph and isinstance(s[3], (int, float))]
            out[ph] = {"samples": len(c),
                       "gfx_mhz_mean": round(sum(c) / len(c), 1) if c else None,
                       "gfx_mhz_min": min(c) if c else None, "gfx_mhz_max": max(c) if c else None,
                       "gfx_mhz_first_last": [c[0], c[-1]] if c else None,
                       "socket_w_mean": round(sum(w) / len(w), 1) if w else None}
            for name in ("MEM", "DF", "SOC"):
                o = [s[4].get(name) for s in self.samples if s[1] == ph]
                o = [x for x in o if isinstance(x, (int, float))]
                if o:
                    out[ph][name.lower() + "_mhz_first_last_min_max"] = [o[0], o[-1], min(o), max(o)]
        return out


def isa_cpi(path: str) -> dict:
    """stage -> mean VALU issue cycles per wave64 instruction of its kernel (isa_mix.json)."""
    try:
        k = json.load(open(path))["kernels"]
    except (OSError, ValueError, KeyError):
        return {}
    return {st: k[name]["cycles_per_valu"] for st, name in STAGE_ISA.items() if name in k}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=700,
                    help="timed steps (700 x ~3.3 ms keeps the timed region above 2 s)")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--blob-mib", type=float, default=256.0)
    ap.add_argument("--n-shards", type=int, default=1000)
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-sample-mib", type=float, default=256.0,
                    help="blob size the CPU restatement encodes+decodes once (default: the full "
                         "256 MiB workload, ~7 s on one core)")
    ap.add_argument("--host-io", choices=["auto", "off"], default="auto",
                    help="also measure the pinned host-in/host-out rate (N=1 only)")
    ap.add_argument("--c3", choices=["auto", "off"], default="auto",
                    help="also time config C3: 128 independent 4 MiB blobs dealt over the ranks, "
                         "one plan per blob, 16 streams per GPU (reported beside the metric)")
    ap.add_argument("--c4", choices=["auto", "off"], default="auto",
                    help="also time config C4: one 4 GiB blob partitioned over the ranks (RCCL "
                         "exchanges), encode + decode from K_p slivers on rank 0")
    ap.add_argument("--host-abi", choices=["auto", "off"], default="auto",
                    help="also time encode_with_metadata / decode through the host-buffer C ABI "
                         "at the metric's size (pageable numpy buffers, N=1 only)")
    ap.add_argument("--quilt", choices=["auto", "off"], default="auto",
                    help="also time a quilt (SURVEY 8(f) 3): 600 blobs, 256 MiB, n=1000; device "
                         "column fill + encode_with_metadata, device-resident (N=1 only)")
    ap.add_argument("--node", choices=["auto", "off"], default="auto",
                    help="also time the storage-node side on the metric's blob (N=1 only): "
                         "verify of every sliver, the recovery-symbol service, one sliver "
                         "recovery (SURVEY 8(f) 1), with the C port's twin in cpu_baseline")
    ap.add_argument("--pmc",default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="per-stage HBM traffic measured by rocprofv3 --pmc (optional)")
    ap.add_argument("--isa", default=os.path.join(ROOT, "profiles", "isa_mix.json"),
                    help="per-kernel VALU issue cycles from the library's ISA (tools/isa_mix.py)")
    ap.add_argument("--overlap", choices=["on", "off"], default="on",
                    help="on: the decode starts on its own stream as soon as the encode's primary "
                         "slivers are written (rs2_encode_device_split_async), beside the "
                         "secondary codecs and the hashing; off: encode then decode in order")
    ap.add_argument("--subsets", choices=["fresh", "fixed"], default="fresh",
                    help="fresh: every step decodes from its own seeded random K_p subset, as a "
                         "client read sees a new sliver subset per blob (the erasure-pattern setup "
                         "is paid every step); fixed: one subset for every step (the reference's "
                         "criterion harness, benches/blob_encoding.rs:98-122)")
    ap.add_argument("--verify", action="store_true", default=True)
    ap.add_argument("--dry-run", nargs="?", const="gloo", default=None, choices=["gloo", "nccl"],
                    help="launcher check without a GPU: ranks join a gloo group and rank 0 "
                         "prints the JSON skeleton with the world size it sees; '--dry-run nccl' "
                         "first runs every rank through the real path's RCCL initialisation "
                         "(init_rccl) and reports how far it got (on a CPU host: the device_id "
                         "check of init_process_group)")
    return ap.parse_args()


def stage_bytes(n, kp, ks, s, blob_len, n_erased_rows, n_present_rows, stages):
    """Algorithmic HBM bytes per launch of each engine stage.
    When the systematic copies are fused into the codec kernels (no enc_sys_transpose /
    dec_copy_present stage), the codec stage also carries those writes."""
    msg = kp * ks * s
    sys_fused = "enc_sys_transpose" not in stages
    dec_fused = "dec_copy_present" not in stages
    # blob copy fused into the systematic-column codec (no enc_blob_copy stage): it also writes
    # the systematic primary slivers
    prim_fused = "enc_blob_copy" not in stages
    tail = msg - (blob_len // (ks * s)) * ks * s
    return {
        "enc_blob_copy": blob_len + msg,
        "enc_tail_rows": 2 * tail,
        "enc_rows_codec": msg + kp * (n - ks) * s,
        "enc_cols_sys_codec": msg + (n - kp) * ks * s + (msg if sys_fused else 0)
                              + (msg if prim_fused else 0),
        "enc_cols_rep_codec": kp * (n - ks) * s + (n - kp) * (n - ks) * s,
        "enc_sys_transpose": 2 * msg,
        # split leaf hashing: enc_leaf_hash_a = the primary slivers' n x K_s leaves (side
        # stream), enc_leaf_hash = the other n x (n - K_s)
        "enc_leaf_hash_a": n * ks * (s + 32),
        "enc_leaf_hash": (n * (n - ks) if "enc_leaf_hash_a" in stages else n * n) * (s + 32),
        "enc_merkle_trees": 2 * n * n * 32 + n * 64,
        "enc_merkle_root": n * 64 + 32,
        "dec_copy_present": 2 * n_present_rows * ks * s,
        "dec_setup": 0,
        "dec_codec": kp * ks * s + n_erased_rows * ks * s
                     + (n_present_rows * ks * s if dec_fused else 0),
    }


# kernel behind each stage (rocprofv3 names; profiles/ summaries list the same kernels)
STAGE_KERNEL = {
    "enc_rows_codec": "rs2_encode_mixed_pipe_kernel<512>",
    "enc_cols_sys_codec": "rs2_encode_shared_pipe_kernel<512>",
    "enc_cols_rep_codec": "rs2_encode_shared_pipe_kernel<512>",
    "enc_sys_transpose": "symbol_copy_kernel",
    "enc_leaf_hash": "leaf_hash_kernel",
    "enc_leaf_hash_a": "leaf_hash_kernel",
    "enc_merkle_trees": "merkle_trees_kernel",
    "enc_merkle_root": "merkle_root_kernel",
    "dec_copy_present": "symbol_copy_kernel",
    "dec_codec": "rs2_decode_kernel<512>",
}


# stages whose span is more than one kernel's duration (rs2_engine.cpp encode_device: the row
# codec is two launches, the blob's whole rows and its zero-padded tail rows)
MULTI_LAUNCH = {"enc_rows_codec"}


def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """`--gpus N` outside torchrun: run this script under torch.distributed.run with N ranks
    (one process per GPU) as a child process -- nothing here has touched the GPU -- and return
    its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def init_rccl(local_rank: int):
    """The multi-GPU run's process group: RCCL (torch's "nccl" backend on ROCm) bound to this
    rank's GPU, rendezvous from the torchrun environment (MASTER_ADDR / MASTER_PORT)."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    return dist


def dry_run(args, world: int, rank: int, local_rank: int) -> None:
    """--dry-run: the launcher contract without a GPU.  With 'nccl', every rank first goes
    through init_rccl exactly as the real run does; on a host without GPUs torch stops it at the
    device_id check (ValueError), which is recorded, on a GPU host it initialises and is torn
    down.  Then the ranks join a gloo group and rank 0 prints one line with what every rank
    saw."""
    import torch.distributed as tdist
    reached = None
    if args.dry_run == "nccl":
        try:
            init_rccl(local_rank)
            reached = f"rccl initialised (world {tdist.get_world_size()})"
            tdist.destroy_process_group()
        except ValueError as e:  # no accelerator: the device_id argument check
            reached = (f"device_id check: {e}" if "device_id" in str(e)
                       else f"ValueError: {e}")
        except Exception as e:  # e.g. no device for this local rank on a host with fewer GPUs
            reached = f"{type(e).__name__}: {e}"
    seen, ranks = 1, [{"rank": rank, "local_rank": local_rank, "nccl": reached}]
    if world > 1:
        tdist.init_process_group("gloo")
        seen = tdist.get_world_size()
        gathered = [None] * seen
        tdist.all_gather_object(gathered, ranks[0])
        ranks = gathered
        tdist.barrier()
    if rank == 0:
        print(json.dumps({"metric": "dry run", "n_gpus": seen, "rank": rank,
                          "backend": args.dry_run, "ranks": ranks}), flush=True)
    if world > 1:
        tdist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        dry_run(args, world, rank, local_rank)
        return

    import numpy as np
    import torch

    torch.cuda.set_device(local_rank)
    import walrus_amd as W
    from walrus_amd import _lib
    _lib.lib().rs2_set_device(local_rank)

    dist = None
    if world > 1:
        dist = init_rccl(local_rank)
        world = dist.get_world_size()  # what RCCL sees (reported as n_gpus)

    n = args.n_shards
    blob_len = int(args.blob_mib * (1 << 20))
    dev = torch.device("cuda", local_rank)
    gen = torch.Generator(device=dev)
    gen.manual_seed(42 + rank)
    blob = torch.randint(0, 256, (blob_len,), dtype=torch.uint8, device=dev, generator=gen)

    # Two sets of plan + sliver / output buffers, used by alternate steps: step k+1's encode
    # (set B) may then overlap step k's decode (set A) without racing it, and step k+2's encode
    # into set A waits only for step k's decode (a step earlier).  --overlap off: one set, encode
    # then decode in order on the main stream.
    n_sets = int(os.environ.get("RS2_BENCH_SETS", "2")) if args.overlap == "on" else 1
    sets = []
    for _ in range(n_sets):
        P_ = W.DevicePlan(n, blob_len)
        inf = P_.info
        sets.append(dict(
            plan=P_,
            primary=torch.empty(n * inf.primary_sliver_len + 256, dtype=torch.uint8, device=dev),
            secondary=torch.empty(n * inf.secondary_sliver_len + 256, dtype=torch.uint8,
                                  device=dev),
            hashes=torch.empty(n * 64, dtype=torch.uint8, device=dev),
            blob_id=torch.empty(32, dtype=torch.uint8, device=dev),
            decoded=torch.empty(blob_len, dtype=torch.uint8, device=dev),
            dec_st=torch.cuda.Stream(dev, priority=int(os.environ.get("RS2_DEC_PRIORITY", "0")))))
    plan = sets[0]["plan"]
    info = plan.info
    kp, ks, s = info.n_primary, info.n_secondary, info.symbol_size
    primary, secondary = sets[0]["primary"], sets[0]["secondary"]
    hashes, blob_id, decoded = sets[0]["hashes"], sets[0]["blob_id"], sets[0]["decoded"]

    # decode from a seeded random subset of K_p primary slivers (random_subset, seed 42): with
    # --subsets fresh a new one every step (warm-up, timed and solo passes), so the decode's
    # per-erasure-pattern plan never repeats; with fixed the first one every step
    rng = np.random.default_rng(42)
    n_sub = (args.warmup + args.steps + SOLO_WARM + SOLO_ITERS) if args.subsets == "fresh" else 1
    subsets = [[int(i) for i in rng.permutation(n)[:kp]] for _ in range(n_sub)]
    idx = subsets[0]
    pl_ = info.primary_sliver_len
    sub_offs = [[i * pl_ for i in sub] for sub in subsets]
    offs = sub_offs[0]
    n_present_all = [sum(1 for i in sub if i < kp) for sub in subsets]
    n_present = int(round(sum(n_present_all) / len(n_present_all)))
    sub_at = [0]

    def next_subset():
        k = sub_at[0] % n_sub
        sub_at[0] += 1
        return subsets[k], sub_offs[k]
    # A/B knobs (tools/stream_ab.sh): RS2_BENCH_MAIN=null|stream (the main-stream work on
    # torch's default stream or on a dedicated one), RS2_BENCH_DEC=2|1 (one decode stream per
    # buffer set, or one shared with per-set events)
    main_mode = os.environ.get("RS2_BENCH_MAIN", "stream")
    dec_mode = int(os.environ.get("RS2_BENCH_DEC", "2"))
    main_prio = int(os.environ.get("RS2_MAIN_PRIORITY", "0"))  # A/B: -1 = high-priority encode
    main_st = (torch.cuda.current_stream(dev) if main_mode == "null"
               else torch.cuda.Stream(dev, priority=main_prio))
    stream = main_st.cuda_stream
    # RS2_BENCH_MAIN=perset (A/B): every buffer set's encode on a stream of its own, so the
    # encodes of consecutive steps may overlap each other too (each still waits for the last
    # decode that read its set)
    for S in sets:
        S["main_st"] = torch.cuda.Stream(dev) if main_mode == "perset" else main_st
    if dec_mode == 1 and n_sets > 1:
        sets[1]["dec_st"] = sets[0]["dec_st"]
    # RS2_BENCH_SPLIT=0 (A/B): the decode waits for the whole encode instead of being released
    # when the primary slivers are final (split encode)
    split_mode = os.environ.get("RS2_BENCH_SPLIT", "1") != "0"
    for S in sets:
        S["dec_done"] = torch.cuda.Event()
        S["dec_done"].record(S["dec_st"])
        S["enc_done"] = torch.cuda.Event()
    counter = [0]
    step_evs = None  # per-step events (RS2_BENCH_STEPTIMES, set before the timed steps)

    def step():
        S = sets[counter[0] % n_sets]
        counter[0] += 1
        idx, offs = next_subset()
        if args.overlap == "on":
            # the decode runs on this set's stream from the moment the primary slivers are final
            # (split encode), beside the secondary codecs and the hashing on the main stream; the
            # main stream first waits for this set's previous decode (two steps back), the last
            # reader of the buffers this encode rewrites
            dst = S["dec_st"]
            S["main_st"].wait_event(S["dec_done"])
            if split_mode:
                S["plan"].encode_split_async(blob.data_ptr(), S["primary"].data_ptr(),
                                             S["secondary"].data_ptr(), S["hashes"].data_ptr(),
                                             S["blob_id"].data_ptr(), S["main_st"].cuda_stream,
                                             dst.cuda_stream)
            else:  # A/B: the decode starts once the whole encode is done
                S["plan"].encode_async(blob.data_ptr(), S["primary"].data_ptr(),
                                       S["secondary"].data_ptr(), S["hashes"].data_ptr(),
                                       S["blob_id"].data_ptr(), S["main_st"].cuda_stream)
                S["enc_done"].record(S["main_st"])
                dst.wait_event(S["enc_done"])
            S["plan"].decode_async("primary", idx, S["primary"].data_ptr(), offs,
                                   S["decoded"].data_ptr(), dst.cuda_stream)
            S["dec_done"].record(dst)
            if step_evs is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(S["main_st"])
                e2 = torch.cuda.Event(enable_timing=True)
                e2.record(dst)
                step_evs.append((e1, e2))
        else:
            S["plan"].encode_async(blob.data_ptr(), S["primary"].data_ptr(),
                                   S["secondary"].data_ptr(), S["hashes"].data_ptr(),
                                   S["blob_id"].data_ptr(), stream)
            S["plan"].decode_async("primary", idx, S["primary"].data_ptr(), offs,
                                   S["decoded"].data_ptr(), stream)

    def profile(on):
        for S in sets:
            S["plan"].profile(on)

    def profile_read():
        acc = {}
        for S in sets:
            for k, (ms, cnt) in S["plan"].profile_read().items():
                a0, c0 = acc.get(k, (0.0, 0))
                acc[k] = (a0 + ms, c0 + cnt)
        return acc

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # The decodes are checked after the timed region (every set's last decode of the timed
    # steps), not between the warm-up and the timed steps: compare kernels and a host round trip
    # there left the first timed steps ~8 % slower (20 timed steps: 84.4-84.8 with vs
    # 86.4-87.2 GiB/s without, profiles/r05/exp/verifywarm/)

    # stage events in the timed steps (the live roofline); RS2_BENCH_PROF=0 (A/B knob) times the
    # steps without them
    prof_timed = os.environ.get("RS2_BENCH_PROF", "1") != "0"
    profile(prof_timed)
    clocks = None
    if os.environ.get("RS2_BENCH_CLOCKS") == "1":
        try:
            clocks = _ClockSampler(local_rank)
            time.sleep(0.05)
        except Exception as e:  # no amdsmi / no permission: the line says so
            clocks = {"error": f"{type(e).__name__}: {e}"}
    if isinstance(clocks, _ClockSampler):
        clocks.phase = "timed"
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    host_ms = []  # host time to issue each step (the issuing thread must stay ahead of the GPU)
    # RS2_BENCH_STEPTIMES=1 (diagnostic): events after each step's encode (main stream) and
    # decode (its stream), reported as offsets from the timed region's start
    step_evs = [] if os.environ.get("RS2_BENCH_STEPTIMES") == "1" else None
    if step_evs is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record(main_st)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        th = time.perf_counter()
        step()
        host_ms.append((time.perf_counter() - th) * 1e3)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    stages = profile_read()
    profile(False)
    if args.verify:
        ok = all(bool(torch.equal(S["decoded"], blob)) for S in sets)
    else:
        ok = None
    # kernel-quality reading: the same stages run one after another (untimed, after the timed
    # region), so each kernel's duration is its own and not stretched by its neighbours.  Each of
    # SOLO_ITERS encode + decode pairs (fresh subsets) is read on its own and every stage's median
    # over them is the solo figure: round 5 took the mean of three pairs right after the timed
    # region and read the decode 10 % above its isolated launch (1.03-1.09 vs 0.94 ms,
    # VERDICT r05 weak #4); tools/solo_probe.py measured that launch at 0.93-0.95 ms in every
    # isolated setting (after an encode, after a 2 GiB flush, back to back, fresh or cached).
    solo_stages = stages
    solo_each = []
    if isinstance(clocks, _ClockSampler):
        clocks.phase = "after_timed"
    # RS2_BENCH_SOLO_PAUSE (seconds, diagnostic): idle time between the timed region and the
    # solo pass
    pause = float(os.environ.get("RS2_BENCH_SOLO_PAUSE", "0"))
    if pause > 0:
        time.sleep(pause)
    if isinstance(clocks, _ClockSampler):
        clocks.phase = "solo_warm"
    if args.overlap == "on":
        # the same pairs unmeasured first, back to back: measured one by one right after the
        # timed region, the first solo decodes ran 10-25 % slow and reached the isolated launch
        # time only after ~8 pairs, with or without a 0.5 s pause and at the same graphics clock
        # (profiles/r06/solo/: RS2_BENCH_CLOCKS samples 2.25-2.39 GHz throughout)
        for _ in range(SOLO_WARM):
            plan.encode_async(blob.data_ptr(), primary.data_ptr(), secondary.data_ptr(),
                              hashes.data_ptr(), blob_id.data_ptr(), stream)
            sidx, soffs = next_subset()
            plan.decode_async("primary", sidx, primary.data_ptr(), soffs, decoded.data_ptr(),
                              stream)
        torch.cuda.synchronize()
    if isinstance(clocks, _ClockSampler):
        clocks.phase = "solo"
    if args.overlap == "on":
        for _ in range(SOLO_ITERS):
            plan.profile(True)
            plan.encode_async(blob.data_ptr(), primary.data_ptr(), secondary.data_ptr(),
                              hashes.data_ptr(), blob_id.data_ptr(), stream)
            sidx, soffs = next_subset()
            plan.decode_async("primary", sidx, primary.data_ptr(), soffs, decoded.data_ptr(),
                              stream)
            torch.cuda.synchronize()
            solo_each.append(plan.profile_read())
            plan.profile(False)
        solo_stages = {}
        for k in solo_each[-1]:
            per = sorted(e[k][0] / max(e[k][1], 1) for e in solo_each if k in e)
            solo_stages[k] = (per[len(per) // 2], 1)

    out = None
    if rank == 0:
        out = _main_line(args, world, n, kp, ks, s, blob_len, n_present, elapsed, stages,
                         solo_stages, ok)
        if step_evs:
            out["step_end_ms"] = [[round(ev0.elapsed_time(a), 3), round(ev0.elapsed_time(b), 3)]
                                  for a, b in step_evs]
        hs = sorted(host_ms)
        out["host_issue_ms_per_step"] = {
            "mean": round(sum(host_ms) / len(host_ms), 4), "median": round(hs[len(hs) // 2], 4),
            "max": round(hs[-1], 4), "first5": [round(x, 3) for x in host_ms[:5]]}
        out["config"]["decode_subsets"] = (
            f"{n_sub} seeded random K_p subsets, one per step (fresh erasure pattern every "
            f"decode; systematic slivers present {min(n_present_all)}..{max(n_present_all)}, "
            f"mean {sum(n_present_all) / len(n_present_all):.1f})" if args.subsets == "fresh"
            else "one seeded random K_p subset for every step")
        if out["roofline"] is not None:
            out["roofline"]["peak_measured_copy_GBs"] = _guarded(lambda: device_copy_gbs(dev))
            if isinstance(clocks, _ClockSampler):
                out["gpu_clocks"] = clocks.summary()
            elif clocks is not None:
                out["gpu_clocks"] = clocks
            if solo_each and "solo" in out["roofline"]:
                dom = out["roofline"]["stage"]
                out["roofline"]["solo"]["ms_each"] = [
                    round(e[dom][0] / max(e[dom][1], 1), 4) for e in solo_each if dom in e]
                out["roofline"]["solo"]["method"] = (
                    f"median of {SOLO_ITERS} encode + decode pairs after the timed region, each "
                    f"read on its own (fresh subsets), after {SOLO_WARM} unmeasured pairs")

    # configs C3 and C4 take every rank (reported beside the metric, never as `value`).  With
    # several ranks a leg that failed on one rank could leave the others waiting in a
    # collective: a watchdog then prints the metric line without it and ends every rank.
    dog = _LegWatchdog(out, rank, LEG_DEADLINE_S) if world > 1 else None
    c3 = c4 = None
    if args.c3 == "auto":
        c3 = _guarded(lambda: c3_leg(n, dev, rank, world, dist))
        if out is not None:
            out["c3_small_blobs"] = c3
    if args.c4 == "auto":
        c4 = _guarded(lambda: c4_leg(n, dev, rank, world, dist))
        if out is not None:
            out["c4_partitioned"] = c4
    if dog:
        dog.cancel()
    if rank != 0:
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    cpu = None
    if args.cpu_baseline == "auto" and world == 1:
        cpu = cpu_baseline(args.cpu_sample_mib, n, node=args.node == "auto",
                           c3_blobs=128 if args.c3 == "auto" else 0)
    c1c2 = None
    if args.c3 == "auto" and world == 1:
        c1c2 = c1_c2_leg(plan, blob, primary, secondary, hashes, blob_id, decoded, idx, n, kp,
                         info.primary_sliver_len, blob_len, stream)
    node = None
    if args.node == "auto" and world == 1:
        node = _guarded(lambda: node_leg(plan, blob, primary, secondary, hashes, blob_id, n, kp,
                                         ks, s, blob_len, stream))
        if node is not None and cpu is not None and cpu.get("node_side"):
            cn = cpu["node_side"]
            node["cpu_twin"] = {k: cn.get(k) for k in ("verify_gibs", "verify_slivers_per_s",
                                                        "recovery_symbols_per_s",
                                                        "recover_sliver_ms", "cores", "ok")}
    if c3 is not None and cpu is not None and cpu.get("c3_twin"):
        ct = cpu["c3_twin"]
        c3["cpu_twin"] = {k: ct.get(k) for k in ("encode_gibs", "cores", "blobs", "wall_s", "ok",
                                                  "sample", "error") if k in ct}
    host_abi = None
    if args.host_abi == "auto" and world == 1:
        host_abi = _guarded(lambda: host_abi_leg(n, blob_len))
    quilt = None
    if args.quilt == "auto" and world == 1:
        quilt = quilt_leg(n, dev)
    host_io = None
    if args.host_io == "auto" and world == 1:
        del primary, secondary, decoded
        sets.clear()
        torch.cuda.empty_cache()
        host_io = host_io_leg(n, blob_len, dev)
    out.update({"cpu_baseline": cpu, "host_io": host_io, "host_abi": host_abi,
                "c1_c2_split": c1c2, "quilt": quilt, "node_side": node})
    print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


LEG_DEADLINE_S = 240.0
SOLO_ITERS = 9  # encode + decode pairs of the solo (kernel-quality) pass
SOLO_WARM = 8   # unmeasured pairs before them


LEG_STALL_EXIT = 3  # exit status of a run whose multi-rank side legs stalled


class _LegWatchdog:
    """Multi-rank side legs with a deadline: if they have not finished after `deadline_s`,
    rank 0 prints the metric line as it stands (pending legs marked) and every rank exits with
    LEG_STALL_EXIT, so a hung collective is a failed run to whoever launched it, not a clean
    one (the measured line is still printed first)."""

    def __init__(self, out, rank, deadline_s):
        import threading
        self._out, self._rank = out, rank
        self._timer = threading.Timer(deadline_s, self._fire)
        self._timer.daemon = True
        self._timer.start()

    def _fire(self):
        if self._rank == 0 and self._out is not None:
            for k in ("c3_small_blobs", "c4_partitioned"):
                if self._out.get(k) is None:
                    self._out[k] = {"error": f"not finished within {LEG_DEADLINE_S:.0f} s"}
            print(json.dumps(self._out), flush=True)
        sys.stdout.flush()
        sys.stderr.write(f"bench: multi-rank side legs stalled for {LEG_DEADLINE_S:.0f} s\n")
        sys.stderr.flush()
        os._exit(LEG_STALL_EXIT)

    def cancel(self):
        self._timer.cancel()


def _main_line(args, world, n, kp, ks, s, blob_len, n_present, elapsed, stages, solo_stages,
               ok):
    """The metric line (rank 0): everything measured on the timed steps."""
    gib = blob_len * args.steps * world / (1 << 30)
    value = gib / elapsed
    # roofline of the dominant kernel: algorithmic bytes per launch / mean launch time
    sb = stage_bytes(n, kp, ks, s, blob_len, kp - n_present, n_present, stages)
    traffic_by_stage = {}
    if os.path.exists(args.pmc):
        try:
            traffic_by_stage = json.load(open(args.pmc))
        except (OSError, ValueError):
            traffic_by_stage = {}

    cpi = isa_cpi(args.isa)

    def roof(st, dom):
        ms, launches = st[dom]
        per_launch_s = ms / 1e3 / max(launches, 1)
        achieved = sb.get(dom, 0) / per_launch_s / 1e9
        out = {"bound": "hbm", "stage": dom, "kernel": STAGE_KERNEL.get(dom, dom),
               "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(achieved / HBM_PEAK_GBS, 5),
               "traffic": traffic_by_stage.get(dom, {}).get("hbm_bytes_per_launch"),
               "ms_per_launch": round(per_launch_s * 1e3, 4)}
        # what actually bounds the codec: vector-instruction issue.  The kernel's wave-VALU
        # instruction count (PMC SQ_INSTS_VALU, --pmc file; fixed for this workload) at its
        # ISA mix's mean issue cycles (isa_mix.json) over what 1,024 SIMDs issue in the live
        # launch time at 2.4 GHz; the flat 2-cycle reading beside it
        vi = traffic_by_stage.get(dom, {}).get("valu_insts_per_launch")
        if vi:
            c = cpi.get(dom, VALU_CYC)
            out["valu_issue_frac"] = round(vi * c / (SIMDS * CLOCK_HZ * per_launch_s), 4)
            out["valu_cycles_per_insn"] = c
            out["valu_issue_frac_2cyc"] = round(vi * VALU_CYC / (SIMDS * CLOCK_HZ * per_launch_s), 4)
        # and the LDS pipe the GF multiplies' table reads go through (PMC SQ_INSTS_LDS at 2 LDS
        # cycles each on 256 CUs): the codec's layers are bound by it
        li = traffic_by_stage.get(dom, {}).get("lds_insts_per_launch")
        if li:
            out["lds_issue_frac"] = round(li * LDS_CYC / (CUS * CLOCK_HZ * per_launch_s), 4)
        return out

    def dominant(st):
        # longest single-kernel stage (the row codec's span holds two launches and a wait on
        # the blob copy, so it is not one kernel's duration)
        cand = {k: v for k, v in st.items() if k in STAGE_KERNEL and k not in MULTI_LAUNCH}
        return max(cand, key=lambda k: cand[k][0] / max(cand[k][1], 1)) if cand else None

    roofline = None
    dom = dominant(stages)
    if dom:
        # the kernel's duration in the timed region (rocprof's average for the same command
        # agrees); with --overlap on it shares the GPU with the encode kernels
        roofline = roof(stages, dom)
        roofline["overlapped"] = args.overlap == "on"
        if args.overlap == "on" and dom in solo_stages:
            roofline["solo"] = {k: v for k, v in roof(solo_stages, dom).items()
                                if k in ("achieved", "frac", "ms_per_launch", "valu_issue_frac",
                                         "valu_issue_frac_2cyc", "lds_issue_frac")}
    enc_bytes = blob_len + n * (ks + kp) * s + 64 * n + 32
    dec_bytes = kp * ks * s + blob_len
    step_s = elapsed / args.steps
    step_roof = {"algorithmic_bytes": enc_bytes + dec_bytes,
                 "achieved_GBs": round((enc_bytes + dec_bytes) / step_s / 1e9, 2),
                 "frac_of_peak": round((enc_bytes + dec_bytes) / step_s / 1e9 / HBM_PEAK_GBS, 5)}
    # the step's vector-issue floor: every stage's VALU wave-instructions per launch (PMC,
    # --pmc file) for the stages this step ran, at 2 cycles each on 1,024 SIMDs at 2.4 GHz --
    # what the step would take if every SIMD issued a VALU instruction every slot
    valu_step = sum(v.get("valu_insts_per_launch") or 0 for k, v in traffic_by_stage.items()
                    if isinstance(v, dict) and k in stages)
    if valu_step:
        # each stage's VALU instructions at its kernel's mean issue cycles (isa_mix.json)
        cyc_step = sum((v.get("valu_insts_per_launch") or 0) * cpi.get(k, VALU_CYC)
                       for k, v in traffic_by_stage.items() if isinstance(v, dict) and k in stages)
        floor_ms = cyc_step / (SIMDS * CLOCK_HZ) * 1e3
        step_roof["valu_insts_per_step"] = int(valu_step)
        step_roof["valu_issue_floor_ms"] = round(floor_ms, 4)
        step_roof["valu_issue_frac"] = round(floor_ms / (step_s * 1e3), 4)
        floor2 = valu_step * VALU_CYC / (SIMDS * CLOCK_HZ) * 1e3
        step_roof["valu_issue_floor_ms_2cyc"] = round(floor2, 4)
        step_roof["valu_issue_frac_2cyc"] = round(floor2 / (step_s * 1e3), 4)
        # per stage: the issue fraction each kernel reaches in its own solo time
        per = {}
        for k, v in traffic_by_stage.items():
            if isinstance(v, dict) and v.get("valu_insts_per_launch") and k in solo_stages:
                ms, launches = solo_stages[k]
                t = ms / 1e3 / max(launches, 1)
                if t > 0 and k not in MULTI_LAUNCH:
                    per[k] = {"cycles_per_insn": cpi.get(k, VALU_CYC),
                              "valu_issue_frac": round(v["valu_insts_per_launch"] *
                                                       cpi.get(k, VALU_CYC) /
                                                       (SIMDS * CLOCK_HZ * t), 4)}
        step_roof["valu_issue_by_stage_solo"] = per
    lds_step = sum(v.get("lds_insts_per_launch") or 0 for k, v in traffic_by_stage.items()
                   if isinstance(v, dict) and k in stages)
    if lds_step:  # the same floor for the CUs' LDS pipes (2 cycles per wave-instruction)
        lfloor_ms = lds_step * LDS_CYC / (CUS * CLOCK_HZ) * 1e3
        step_roof["lds_insts_per_step"] = int(lds_step)
        step_roof["lds_issue_floor_ms"] = round(lfloor_ms, 4)
        step_roof["lds_issue_frac"] = round(lfloor_ms / (step_s * 1e3), 4)

    out = {
        "metric": "Red Stuff encode+decode GiB/s (device-resident), 256 MiB blob, n_shards=1000",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic (seeded uniform random bytes, torch.Generator seed 42+rank)",
        "config": {
            "workload": ("encode_with_metadata + primary decode from a fresh seeded random K_p "
                         "subset per step" if args.subsets == "fresh" else
                         "encode_with_metadata + primary decode from a seeded random K_p subset"),
            "n_shards": n, "blob_bytes": blob_len, "n_primary": kp, "n_secondary": ks,
            "symbol_size": s, "decode_axis": "primary", "decode_present_systematic": n_present,
            "parallelism": f"independent blobs x{world}",
        },
        "roofline": roofline,
        "step_roofline": step_roof,
        "stages_ms_per_step": {k: round(v[0] / max(v[1], 1), 4) for k, v in stages.items()},
        "stages_ms_solo": ({k: round(v[0] / max(v[1], 1), 4) for k, v in solo_stages.items()}
                           if args.overlap == "on" else None),
        "overlap": args.overlap,
        "cpu_baseline": None,
        "host_io": None,
        "host_abi": None,
        "c1_c2_split": None,
        "c3_small_blobs": None,
        "c4_partitioned": None,
        "quilt": None,
        "node_side": None,
        "decode_roundtrip_ok": ok,
    }
    return out


def host_io_leg(n: int, blob_len: int, dev, blobs: int = 6):
    """PCIe-inclusive rates (never `value`): the blob starts in pinned host memory and the
    slivers / decoded blob end there (north_star: "the rate including pinned hipMemcpyAsync to
    and from the GPU").  Three streams overlap H2D of blob i+1, the engine on blob i and D2H
    of blob i-1; two device slots (one plan each, so no re-binding between blobs).
    Returns GiB/s of blob bytes for: encode+decode (the metric's step), encode only
    (slivers + metadata out), compute_metadata (blob in, 64n+32 B out)."""
    import numpy as np
    import torch
    import walrus_amd as W

    plans = [W.DevicePlan(n, blob_len) for _ in range(2)]
    info = plans[0].info
    kp, pl, sl = info.n_primary, info.primary_sliver_len, info.secondary_sliver_len
    g = torch.Generator().manual_seed(7)
    h_blob = torch.randint(0, 256, (blob_len,), dtype=torch.uint8, generator=g).pin_memory()
    # decode input: K_p primary slivers (seeded subset), as they arrive from storage nodes
    idx = [int(i) for i in np.random.default_rng(42).permutation(n)[:kp]]
    h_sliv = torch.empty(kp * pl, dtype=torch.uint8).pin_memory()
    slots = []
    for _ in range(2):
        slots.append(dict(
            d_blob=torch.empty(blob_len, dtype=torch.uint8, device=dev),
            d_prim=torch.empty(n * pl + 256, dtype=torch.uint8, device=dev),
            d_sec=torch.empty(n * sl + 256, dtype=torch.uint8, device=dev),
            d_hash=torch.empty(n * 64, dtype=torch.uint8, device=dev),
            d_bid=torch.empty(32, dtype=torch.uint8, device=dev),
            d_sliv=torch.empty(kp * pl, dtype=torch.uint8, device=dev),
            d_dec=torch.empty(blob_len, dtype=torch.uint8, device=dev),
            h_prim=torch.empty(n * pl, dtype=torch.uint8).pin_memory(),
            h_sec=torch.empty(n * sl, dtype=torch.uint8).pin_memory(),
            h_hash=torch.empty(n * 64 + 32, dtype=torch.uint8).pin_memory(),
            h_dec=torch.empty(blob_len, dtype=torch.uint8).pin_memory(),
            free=torch.cuda.Event(), ready=torch.cuda.Event(), done=torch.cuda.Event()))
    # the decode input slivers are real encoder output of h_blob
    s0 = slots[0]
    s0["d_blob"].copy_(h_blob)
    plans[0].encode_async(s0["d_blob"].data_ptr(), s0["d_prim"].data_ptr(), s0["d_sec"].data_ptr(),
                          s0["d_hash"].data_ptr(), s0["d_bid"].data_ptr(),
                          torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    for j, i in enumerate(idx):
        h_sliv[j * pl:(j + 1) * pl].copy_(s0["d_prim"][i * pl:(i + 1) * pl])
    offs = [j * pl for j in range(kp)]
    st_in, st_run, st_out = (torch.cuda.Stream(dev) for _ in range(3))

    def run(mode: str, count: int) -> float:
        for sl_ in slots:
            sl_["free"].record(st_out)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for b in range(count):
            k = b % 2
            S, P = slots[k], plans[k]
            with torch.cuda.stream(st_in):
                st_in.wait_event(S["free"])
                S["d_blob"].copy_(h_blob, non_blocking=True)
                if mode == "encdec":
                    S["d_sliv"].copy_(h_sliv, non_blocking=True)
                S["ready"].record(st_in)
            st_run.wait_event(S["ready"])
            P.encode_async(S["d_blob"].data_ptr(), S["d_prim"].data_ptr(), S["d_sec"].data_ptr(),
                           S["d_hash"].data_ptr(), S["d_bid"].data_ptr(), st_run.cuda_stream)
            if mode == "encdec":
                P.decode_async("primary", idx, S["d_sliv"].data_ptr(), offs,
                               S["d_dec"].data_ptr(), st_run.cuda_stream)
            S["done"].record(st_run)
            with torch.cuda.stream(st_out):
                st_out.wait_event(S["done"])
                if mode != "meta":
                    S["h_prim"].copy_(S["d_prim"][:n * pl], non_blocking=True)
                    S["h_sec"].copy_(S["d_sec"][:n * sl], non_blocking=True)
                S["h_hash"][:n * 64].copy_(S["d_hash"], non_blocking=True)
                S["h_hash"][n * 64:].copy_(S["d_bid"], non_blocking=True)
                if mode == "encdec":
                    S["h_dec"].copy_(S["d_dec"], non_blocking=True)
                S["free"].record(st_out)
        torch.cuda.synchronize(dev)
        return count * blob_len / (1 << 30) / (time.perf_counter() - t0)

    run("encdec", 2)  # warm-up (pinned pages, plan binding)
    out = {"encode_decode_gibs": round(run("encdec", blobs), 3),
           "encode_gibs": round(run("enc", blobs), 3),
           "compute_metadata_gibs": round(run("meta", blobs), 3)}
    ok = bool(torch.equal(slots[(blobs - 1) % 2]["h_dec"], h_blob))
    out.update({"blobs": blobs, "decode_roundtrip_ok": ok,
                "note": "pinned host buffers, 3 streams (H2D / engine / D2H), 2 device slots; "
                        "encode D2H = n*(K_s+K_p)*s sliver bytes + metadata"})
    del slots, plans
    torch.cuda.empty_cache()
    return out


def c1_c2_leg(plan, blob, primary, secondary, hashes, blob_id, decoded, idx, n, kp, pl,
              blob_len, stream, reps: int = 10):
    """BASELINE configs C1 and C2 on their own (reported beside the metric): encode_with_metadata
    alone, and the primary decode alone from (i) the bench's random K_p subset, (ii) a fresh
    random subset every call and (iii) the worst case, slivers K_p..2K_p (no systematic sliver
    present), device-resident, one stream."""
    import numpy as np
    import torch

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    gib = blob_len / (1 << 30)
    enc = timed(lambda: plan.encode_async(blob.data_ptr(), primary.data_ptr(),
                                          secondary.data_ptr(), hashes.data_ptr(),
                                          blob_id.data_ptr(), stream))
    out = {"c1_encode_gibs": round(gib / enc, 3), "c1_encode_ms": round(enc * 1e3, 4)}
    # BlobEncoder::compute_metadata on the device blob (the criterion harness times it on its
    # own, benches/blob_encoding.rs:44-50; the upload relay's call): pair hashes + BlobId only
    m_hashes = torch.empty_like(hashes)
    m_id = torch.empty_like(blob_id)
    cm = timed(lambda: plan.compute_metadata_async(blob.data_ptr(), m_hashes.data_ptr(),
                                                   m_id.data_ptr(), stream))
    out["c1_compute_metadata_gibs"] = round(gib / cm, 3)
    out["c1_compute_metadata_ms"] = round(cm * 1e3, 4)
    out["c1_compute_metadata_ok"] = bool(torch.equal(m_hashes, hashes) and
                                         torch.equal(m_id, blob_id))
    worst = list(range(kp, 2 * kp))
    for name, sel in (("c2_decode_random", idx), ("c2_decode_worst", worst)):
        offs = [i * pl for i in sel]
        decoded.zero_()
        dt = timed(lambda: plan.decode_async("primary", sel, primary.data_ptr(), offs,
                                             decoded.data_ptr(), stream))
        out[name + "_gibs"] = round(gib / dt, 3)
        out[name + "_ms"] = round(dt * 1e3, 4)
        out[name + "_ok"] = bool(torch.equal(decoded, blob))
    # the same decode with a fresh erasure pattern per call (a client read: a new sliver
    # subset per blob), so the per-pattern setup (locator FWHT, block mixing, table uploads and
    # the multiplier-table kernel) is in every call: the twin of c2_decode_random
    frng = np.random.default_rng(4242)
    fresh = [[int(i) for i in frng.permutation(n)[:kp]] for _ in range(reps + 1)]
    it = iter(fresh)

    def fresh_decode():
        sel = next(it)
        plan.decode_async("primary", sel, primary.data_ptr(), [i * pl for i in sel],
                          decoded.data_ptr(), stream)
    decoded.zero_()
    dt = timed(fresh_decode)
    out["c2_decode_random_fresh_gibs"] = round(gib / dt, 3)
    out["c2_decode_random_fresh_ms"] = round(dt * 1e3, 4)
    out["c2_decode_random_fresh_ok"] = bool(torch.equal(decoded, blob))
    out["c2_fresh_vs_cached"] = round(out["c2_decode_random_fresh_ms"] /
                                      out["c2_decode_random_ms"], 4)
    # C2 with the consistency checks on the device (benches/blob_encoding.rs:81-99 times
    # decode_and_verify with each ConsistencyCheckType): rs2_decode_and_verify_device from the
    # same device slivers; the call returns with the verdict (synchronous), so it is timed as is
    torch.cuda.synchronize()
    h_meta = bytes(hashes.cpu().numpy())
    h_id = bytes(blob_id.cpu().numpy())
    for name, sel in (("random", idx), ("worst", worst)):
        offs = [i * pl for i in sel]
        for check in ("skip", "default", "strict"):
            decoded.zero_()
            dt = timed(lambda: plan.decode_and_verify("primary", sel, primary.data_ptr(), offs,
                                                      h_meta, h_id, check, decoded.data_ptr(),
                                                      stream))
            key = f"c2_verify_{check}_{name}"
            out[key + "_gibs"] = round(gib / dt, 3)
            out[key + "_ms"] = round(dt * 1e3, 4)
            out[key + "_ok"] = bool(torch.equal(decoded, blob))
    # C2 through the host API (decode / decode_and_verify with host slivers, pageable buffers:
    # the H2D of the K_p slivers is inside the time), Skip / Default / Strict consistency checks
    import walrus_amd as W
    torch.cuda.synchronize()
    plan.encode_async(blob.data_ptr(), primary.data_ptr(), secondary.data_ptr(),
                      hashes.data_ptr(), blob_id.data_ptr(), stream)
    torch.cuda.synchronize()
    s = plan.info.symbol_size
    host = primary[:n * pl].view(n, pl)[torch.tensor(idx, device=primary.device)].cpu().numpy()
    slivers = [W.SliverData(W.Symbols(host[j].tobytes(), s), i, W.PRIMARY)
               for j, i in enumerate(idx)]
    h = bytes(hashes.cpu().numpy())
    meta = W.VerifiedBlobMetadataWithId(
        W.BlobId(bytes(blob_id.cpu().numpy())),
        W.BlobMetadata([(h[64 * i:64 * i + 32], h[64 * i + 32:64 * i + 64]) for i in range(n)],
                       blob_len))
    cfg = W.ReedSolomonEncodingConfig(n)
    want = bytes(blob.cpu().numpy())
    for check in ("skip", "default", "strict"):
        got = cfg.decode_and_verify(meta, slivers, check)  # warm (plan build)
        t0 = time.perf_counter()
        got = cfg.decode_and_verify(meta, slivers, check)
        dt = time.perf_counter() - t0
        out[f"c2_host_{check}_gibs"] = round(gib / dt, 3)
        out[f"c2_host_{check}_ok"] = got == want
    return out


def node_leg(plan, blob, primary, secondary, hashes, blob_id, n, kp, ks, s, blob_len, stream,
             reps: int = 10):
    """The storage-node side of the path, device-resident on the C1 blob's
    slivers (encoded by `plan` into primary / secondary just before):
      * verify: SliverData::verify of all n primary and n secondary slivers -- expand each on
        the orthogonal axis, n leaf hashes, the n-leaf root, compared with the metadata
        (walrus-service node.rs:2615-2633, slivers.rs:100-135); two rs2_verifier launches;
      * recovery symbols: n requests, request i = primary sliver i's expanded symbol
        (i*7+3) mod n with its Merkle proof (recovery_symbol_service.rs:161-235,
        slivers.rs:180-213) -- the same requests the CPU twin (cpu_baseline.node_side) times;
      * recover: recover_sliver_or_generate_inconsistency_proof (slivers.rs:341-379,
        request_futures.rs:436-497) of one primary sliver from K_s verified recovery symbols
        held in host memory, as they arrive from other nodes, through the public API (decode
        on the GPU + verify against the metadata): latency per call.
    Parity: roots equal the metadata's hashes; every recovery symbol's proof recomputes its
    source sliver's hash and the symbol equals the sliver byte it names where the encode
    stored it; the recovered sliver equals the encoded one."""
    import numpy as np
    import torch
    import walrus_amd as W
    from walrus_amd import recovery as R

    dev = primary.device
    torch.cuda.synchronize()
    plan.encode_async(blob.data_ptr(), primary.data_ptr(), secondary.data_ptr(),
                      hashes.data_ptr(), blob_id.data_ptr(), stream)
    torch.cuda.synchronize()
    pl, sl = ks * s, kp * s
    vp = W.SliverVerifier(n, s, W.PRIMARY)
    vs = W.SliverVerifier(n, s, W.SECONDARY)
    roots_p = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    roots_s = torch.empty(n * 32, dtype=torch.uint8, device=dev)

    def timed(fn, k=reps):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k

    def verify():
        vp.roots_async(n, primary.data_ptr(), roots_p.data_ptr(), stream)
        vs.roots_async(n, secondary.data_ptr(), roots_s.data_ptr(), stream)
    dt = timed(verify)
    hv = hashes[:n * 64].view(n, 64)
    ok_v = bool(torch.equal(roots_p.view(n, 32), hv[:, :32]) and
                torch.equal(roots_s.view(n, 32), hv[:, 32:].flip(0)))
    vbytes = n * (ks + kp) * s
    out = {"node_verify_gibs": round(vbytes / dt / (1 << 30), 3),
           "node_verify_slivers_per_s": round(2 * n / dt, 1),
           "node_verify_ms": round(dt * 1e3, 4), "node_verify_ok": ok_v,
           "node_verify_sample": f"all {n} primary + {n} secondary slivers "
                                 f"({vbytes / 1e9:.3f} GB), one launch per axis"}

    # recovery-symbol service: n requests, source primary sliver i, symbol (i*7+3) mod n
    L = R.path_length(n)
    targets = [(i * 7 + 3) % n for i in range(n)]
    d_sym = torch.empty(n * s, dtype=torch.uint8, device=dev)
    d_prf = torch.empty(n * L * 32, dtype=torch.uint8, device=dev)
    dt = timed(lambda: vp.recovery_symbols_async(n, primary.data_ptr(), targets, d_sym.data_ptr(),
                                                 d_prf.data_ptr(), 0, stream))
    syms = d_sym.cpu().numpy().reshape(n, s)
    prfs = d_prf.cpu().numpy().reshape(n, L * 32)
    hh = hashes[:n * 64].cpu().numpy().reshape(n, 64)
    roots = R.compute_roots([R.MerkleProof([bytes(prfs[i, 32 * l:32 * l + 32]) for l in range(L)])
                             for i in range(n)], [bytes(syms[i]) for i in range(n)], targets)
    ok_r = all(roots[i] == bytes(hh[i, :32]) for i in range(n))
    prim_h = primary[:n * pl].view(n, ks, s)
    sec_h = secondary[:n * sl].view(n, kp, s)
    for i in range(0, n, 37):  # the stored symbols among the requests
        t = targets[i]
        want = prim_h[i, t] if t < ks else (sec_h[t, i] if i < kp else None)
        if want is not None:
            ok_r &= bytes(want.cpu().numpy()) == bytes(syms[i])
    out.update({"recovery_symbols_per_s": round(n / dt, 1),
                "recovery_symbols_ms": round(dt * 1e3, 4), "recovery_symbols_ok": bool(ok_r),
                "recovery_symbols_sample": f"{n} requests (symbol + {L}-node proof), one launch"})

    # recover one primary sliver from K_s recovery symbols (from secondary slivers n-1, n-2, ...
    # whose expansions' symbol `target` the service returns), host-in, verified on the way out
    target = 131
    srcs = list(range(n - 1, n - 1 - ks, -1))
    d_src = secondary[:n * sl].view(n, sl)[torch.tensor(srcs, device=dev)].contiguous()
    d_sym2 = torch.empty(ks * s, dtype=torch.uint8, device=dev)
    d_prf2 = torch.empty(ks * L * 32, dtype=torch.uint8, device=dev)
    vs.recovery_symbols_async(ks, d_src.data_ptr(), [target] * ks, d_sym2.data_ptr(),
                              d_prf2.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    s2 = d_sym2.cpu().numpy().reshape(ks, s)
    p2 = d_prf2.cpu().numpy().reshape(ks, L * 32)
    rsyms = [R.RecoverySymbol(W.PRIMARY, c, bytes(s2[q]),
                              R.MerkleProof([bytes(p2[q, 32 * l:32 * l + 32]) for l in range(L)]))
             for q, c in enumerate(srcs)]
    h = bytes(hh.tobytes())
    meta = W.BlobMetadata([(h[64 * i:64 * i + 32], h[64 * i + 32:64 * i + 64]) for i in range(n)],
                          blob_len)
    cfg = W.ReedSolomonEncodingConfig(n)
    got = R.recover_sliver_or_generate_inconsistency_proof(rsyms, target, meta, cfg, W.PRIMARY)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        got = R.recover_sliver_or_generate_inconsistency_proof(rsyms, target, meta, cfg,
                                                               W.PRIMARY)
        times.append(time.perf_counter() - t0)
    ok_s = (isinstance(got, W.SliverData) and
            got.symbols.data == bytes(primary[target * pl:(target + 1) * pl].cpu().numpy()))
    out.update({"recover_sliver_ms": round(sorted(times)[len(times) // 2] * 1e3, 4),
                "recover_sliver_ok": bool(ok_s),
                "recover_sliver_sample": f"primary sliver {target} from K_s = {ks} verified "
                                         "recovery symbols in host memory (public API: decode "
                                         "+ verify against the metadata), median of "
                                         f"{reps} calls"})
    return out


def quilt_leg(n: int, dev, blobs: int = 600, total_mib: int = 256, reps: int = 10):
    """Quilt V1 encode, device-resident: the serialized payload stream and the column table are
    in HBM; one step = the device column fill (rs2_quilt_layout_device_async) + the quilt's
    encode_with_metadata.  GiB/s of quilt bytes (K_p*K_s*s), checked against the host layout."""
    import numpy as np
    import torch
    import walrus_amd as W
    from walrus_amd import quilt as Q

    rng = np.random.default_rng(11)
    per = (total_mib << 20) // blobs
    items = [Q.QuiltStoreBlob(rng.integers(0, 256, int(per * rng.uniform(0.5, 1.0)),
                                           dtype=np.uint8).tobytes(),
                              f"blob-{i:04d}.bin", {"kind": "bench"} if i % 3 == 0 else {})
             for i in range(blobs)]
    cfg = W.ReedSolomonEncodingConfig(n)
    enc = Q.QuiltEncoderV1(cfg, items)
    lay = enc.layout()
    t0 = time.perf_counter()
    host_quilt = enc.construct_quilt()
    host_layout_s = time.perf_counter() - t0
    d_pay = torch.from_numpy(np.frombuffer(lay.payload, dtype=np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(lay.col_off).to(dev)
    d_len = torch.from_numpy(lay.col_len.astype(np.int32)).to(dev)
    d_q = torch.empty(lay.quilt_len, dtype=torch.uint8, device=dev)
    plan = W.DevicePlan(n, lay.quilt_len)
    info = plan.info
    prim = torch.empty(n * info.primary_sliver_len + 256, dtype=torch.uint8, device=dev)
    sec = torch.empty(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
    meta = torch.empty(n * 64 + 32, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def step():
        Q.quilt_layout_device_async(lay, d_pay.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                    d_q.data_ptr(), st)
        plan.encode_async(d_q.data_ptr(), prim.data_ptr(), sec.data_ptr(), meta.data_ptr(),
                          meta[n * 64:].data_ptr(), st)

    step()
    torch.cuda.synchronize()
    ok = bytes(d_q.cpu().numpy()) == host_quilt.data
    layout_ms = 0.0
    t0 = time.perf_counter()
    for _ in range(reps):
        ev[0].record()
        Q.quilt_layout_device_async(lay, d_pay.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                    d_q.data_ptr(), st)
        ev[1].record()
        plan.encode_async(d_q.data_ptr(), prim.data_ptr(), sec.data_ptr(), meta.data_ptr(),
                          meta[n * 64:].data_ptr(), st)
        ev[2].record()
        torch.cuda.synchronize()
        layout_ms += ev[0].elapsed_time(ev[1])
    dt = (time.perf_counter() - t0) / reps
    qb = lay.quilt_len
    out = {"quilt_encode_gibs": round(qb / (1 << 30) / dt, 3), "ms_per_quilt": round(dt * 1e3, 4),
           "layout_ms": round(layout_ms / reps, 4),
           "layout_GBs": round(2 * qb / (layout_ms / reps / 1e3) / 1e9, 1),
           "host_layout_ms": round(host_layout_s * 1e3, 1),
           "blobs": blobs, "quilt_bytes": qb, "payload_bytes": len(lay.payload),
           "symbol_size": lay.symbol_size, "columns_used": int(lay.index.quilt_patches[-1].end_index),
           "device_layout_matches_host": ok,
           "note": "device-resident payload stream + column table; layout kernel + "
                   "encode_with_metadata per quilt, one stream, synchronised per quilt"}
    del d_pay, d_q, prim, sec
    torch.cuda.empty_cache()
    return out


def _guarded(fn):
    """Run a side leg; a failure is reported in its JSON slot instead of losing the line."""
    try:
        return fn()
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        return {"error": f"{type(e).__name__}: {e}"}


def _timed_max(fn, dist, dev, reps: int):
    """Best of `reps` runs of fn(), each bracketed by barrier + synchronize and taken as the
    max over ranks."""
    import torch
    best = None
    for _ in range(reps):
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        if dist:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        best = dt if best is None else min(best, dt)
    return best


def c3_leg(n: int, dev, rank: int, world: int, dist, total_blobs: int = 128,
           streams_per_gpu: int = 16, reps: int = 5):
    """BASELINE config C3: 128 independent 4 MiB blobs, encode_with_metadata, dealt round-robin
    over the ranks (walrus_amd.dist.shard_blobs; the reference's rayon over blobs,
    walrus-sdk/src/node_client.rs:3182).  One plan per blob, 16 streams per GPU, all
    device-resident; no collective on the data path -- the 32-byte BlobIds are all-gathered
    once after the timed region and checked against a serial re-encode on each rank."""
    import torch
    import walrus_amd as W
    from walrus_amd.dist import shard_blobs

    blob_len = 4 << 20
    mine = shard_blobs(total_blobs, rank, world)
    plans = [W.DevicePlan(n, blob_len) for _ in mine]
    info = plans[0].info
    bufs = []
    for b in mine:
        g = torch.Generator(device=dev)
        g.manual_seed(1000 + b)
        bufs.append(dict(
            blob=torch.randint(0, 256, (blob_len,), dtype=torch.uint8, device=dev, generator=g),
            prim=torch.empty(n * info.primary_sliver_len + 256, dtype=torch.uint8, device=dev),
            sec=torch.empty(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev),
            hashes=torch.empty(n * 64, dtype=torch.uint8, device=dev),
            bid=torch.empty(32, dtype=torch.uint8, device=dev)))
    streams = [torch.cuda.Stream(dev) for _ in range(min(streams_per_gpu, len(mine)))]

    def batch():
        for k, (P, b) in enumerate(zip(plans, bufs)):
            P.encode_async(b["blob"].data_ptr(), b["prim"].data_ptr(), b["sec"].data_ptr(),
                           b["hashes"].data_ptr(), b["bid"].data_ptr(),
                           streams[k % len(streams)].cuda_stream)

    batch()
    best_streams = _timed_max(batch, dist, dev, reps)
    # the same blobs through ONE batched call (rs2_encode_batch_device_async: one launch per
    # stage over every blob of this rank), from one strided copy of the blobs
    nb = len(mine)
    pl, sl = info.primary_sliver_len, info.secondary_sliver_len
    bstride = blob_len
    bat = dict(blob=torch.stack([b["blob"] for b in bufs]),
               prim=torch.empty((nb, n * pl), dtype=torch.uint8, device=dev),
               sec=torch.empty((nb, n * sl), dtype=torch.uint8, device=dev),
               hashes=torch.empty((nb, n * 64), dtype=torch.uint8, device=dev),
               bid=torch.empty((nb, 32), dtype=torch.uint8, device=dev))
    bplan = W.DevicePlan(n, blob_len)
    bst = torch.cuda.Stream(dev)

    def batched():
        bplan.encode_batch_async(nb, bat["blob"].data_ptr(), bstride, None, bat["prim"].data_ptr(),
                                 n * pl, bat["sec"].data_ptr(), n * sl, bat["hashes"].data_ptr(),
                                 bat["bid"].data_ptr(), bst.cuda_stream)

    batched()
    best = _timed_max(batched, dist, dev, reps)
    torch.cuda.synchronize(dev)
    batch_ok = all(bool(torch.equal(bat["bid"][j], b["bid"])) and
                   bool(torch.equal(bat["hashes"][j], b["hashes"])) for j, b in enumerate(bufs))
    # every BlobId equals a serial re-encode on one stream, then all ranks' ids are gathered
    ref = torch.empty(n * 64 + 32, dtype=torch.uint8, device=dev)
    st0 = torch.cuda.current_stream(dev).cuda_stream
    ok = True
    for b in bufs:
        plans[0].encode_async(b["blob"].data_ptr(), bufs[0]["prim"].data_ptr(),
                              bufs[0]["sec"].data_ptr(), ref[:n * 64].data_ptr(),
                              ref[n * 64:].data_ptr(), st0)
        torch.cuda.synchronize(dev)
        ok &= bool(torch.equal(ref[:n * 64], b["hashes"])) and bool(torch.equal(ref[n * 64:], b["bid"]))
    n_ids = total_blobs
    if dist:
        okt = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())
        per = -(-total_blobs // world)
        loc = torch.zeros(per * 32, dtype=torch.uint8, device=dev)
        for j, b in enumerate(bufs):
            loc[j * 32:(j + 1) * 32].copy_(b["bid"])
        parts = [torch.empty_like(loc) for _ in range(world)]
        dist.all_gather(parts, loc)
        n_ids = sum(len(shard_blobs(total_blobs, r, world)) for r in range(world))
    out = {"encode_gibs": round(total_blobs * blob_len / (1 << 30) / best, 3),
           "encode_gibs_streams": round(total_blobs * blob_len / (1 << 30) / best_streams, 3),
           "blobs": total_blobs, "blobs_per_rank": len(mine), "ranks": world,
           "blob_ids_gathered": n_ids, "serial_reencode_matches": ok,
           "batched_matches_streams": batch_ok,
           "blob_bytes": blob_len, "symbol_size": info.symbol_size,
           "ms_per_batch": round(best * 1e3, 3),
           "ms_per_batch_streams": round(best_streams * 1e3, 3),
           "note": "encode_with_metadata of every blob of the rank: encode_gibs = one batched call "
                   "(rs2_encode_batch_device_async, one launch per stage); encode_gibs_streams = "
                   "one plan per blob over 16 streams; device-resident, "
                   f"best of {reps}, max over ranks; BlobIds all-gathered afterwards"}
    del plans, bufs, bat, bplan
    torch.cuda.empty_cache()
    return out


def c4_leg(n: int, dev, rank: int, world: int, dist, blob_len: int = 4 << 30, reps: int = 3):
    """BASELINE config C4: one 4 GiB blob, encode_with_metadata row/column-partitioned over the
    ranks (walrus_amd.partition: row code on each rank's rows, RCCL all-to-all into column
    ownership, column code + leaf hashes + column trees, all-to-all of leaf digests, row
    trees, RCCL all-to-all of the primary slivers' symbols into sliver-pair ownership, local
    secondary-sliver gather, all-gather of the roots: every rank ends with its assembled sliver
    pairs, inside the timed encode), then BlobDecoder::decode from K_p primary slivers held by
    rank 0 (RCCL scatter of column ranges, per-rank column decodes, RCCL gather of the decoded
    columns).  Timed max over ranks; the decoded blob is checked on rank 0 and every rank's
    BlobId must agree."""
    import numpy as np
    import torch
    from walrus_amd import partition as P

    part = P.Partition.for_blob(n, blob_len, world)
    ops = P.DeviceOps()
    ex = P.DistExchange() if dist else P.LocalExchange()
    g = torch.Generator(device=dev)
    g.manual_seed(404)  # every rank generates the same blob and keeps its own rows
    blob = torch.randint(0, 256, (blob_len,), dtype=torch.uint8, device=dev, generator=g)
    rows = P.rows_of_blob(part, blob, rank)
    if rank != 0:
        del blob
        blob = None
    res = {}

    def enc():
        res["enc"] = P.encode_distributed(part, rows, ops, ex, dev)

    enc()
    enc_s = _timed_max(enc, dist, dev, reps)
    e = res["enc"]
    # the K_p received primary slivers on rank 0, gathered from the ranks whose sliver pairs
    # they are (setup, untimed: stands for slivers arriving from storage nodes)
    idx = [int(i) for i in np.random.default_rng(42).permutation(n)[:part.kp]]
    slivers = P.collect_primary(part, e, idx, ex)

    def dec():
        res["dec"] = P.decode_from_slivers(part, slivers, idx, ops, ex, dev)

    dec()
    dec_s = _timed_max(dec, dist, dev, reps)
    ok = bool(torch.equal(res["dec"], blob)) if rank == 0 else True
    bids = ex.all_gather(e.blob_id)
    same = bool((bids.view(world, 32) == e.blob_id.view(1, 32)).all())
    if dist:
        t = torch.tensor([1 if (ok and same) else 0], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        ok = bool(t.item())
    else:
        ok = ok and same
    gib = blob_len / (1 << 30)
    out = {"encode_gibs": round(gib / enc_s, 3), "decode_gibs": round(gib / dec_s, 3),
           "encode_decode_gibs": round(gib / (enc_s + dec_s), 3),
           "encode_ms": round(enc_s * 1e3, 3), "decode_ms": round(dec_s * 1e3, 3),
           "ranks": world, "blob_bytes": blob_len, "symbol_size": part.s,
           "decode_roundtrip_and_blob_ids_ok": ok,
           "note": "partitioned encode (RCCL all-to-all x3 + all-gather; each rank ends with its "
                   "assembled sliver pairs) and decode from K_p "
                   f"primary slivers on rank 0 (RCCL scatter + gather); best of {reps}, max "
                   "over ranks, device-resident"}
    del res, rows, slivers, blob
    torch.cuda.empty_cache()
    return out


def host_abi_leg(n: int, blob_len: int, reps: int = 3):
    """C1 / C2 through the host-buffer C ABI a Rust caller binds (include/walrus_rs2.h):
    rs2_encode_with_metadata (blob in, 2n slivers + metadata out) and rs2_decode_blob (K_p
    primary slivers in, blob out), pageable numpy buffers, the engine's pinned staging ring
    inside the time.  Buffers are reused across calls (pre-faulted), as a service would."""
    import ctypes
    import numpy as np
    import walrus_amd as W
    from walrus_amd import _lib

    L = _lib.lib()
    cfg = W.ReedSolomonEncodingConfig(n)
    plan = cfg._plan(blob_len)
    info = plan.info
    pl, sl, kp = info.primary_sliver_len, info.secondary_sliver_len, info.n_primary
    blob = np.random.default_rng(8).integers(0, 256, blob_len, dtype=np.uint8)
    prim = np.ones((n, pl), dtype=np.uint8)
    sec = np.ones((n, sl), dtype=np.uint8)
    hashes = np.zeros(n * 64, dtype=np.uint8)
    bid = np.zeros(32, dtype=np.uint8)
    pp = (ctypes.c_void_p * n)(*[prim[i].ctypes.data for i in range(n)])
    sp = (ctypes.c_void_p * n)(*[sec[i].ctypes.data for i in range(n)])
    idx = [int(i) for i in np.random.default_rng(42).permutation(n)[:kp]]
    ia = (ctypes.c_uint16 * kp)(*idx)
    sa = (ctypes.c_void_p * kp)(*[prim[i].ctypes.data for i in idx])
    la = (ctypes.c_uint64 * kp)(*([pl] * kp))
    out = np.ones(blob_len, dtype=np.uint8)

    def encode():
        rc = L.rs2_encode_with_metadata(plan.handle, blob.ctypes.data, pp, sp, hashes.ctypes.data,
                                        bid.ctypes.data)
        assert rc == 0, _lib.last_error()

    def decode():
        rc = L.rs2_decode_blob(plan.handle, 0, kp, ia, sa, la, None, out.ctypes.data)
        assert rc == 0, _lib.last_error()

    def best(fn):
        fn()
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            t.append(time.perf_counter() - t0)
        return min(t)

    te, td = best(encode), best(decode)
    ok = bool(np.array_equal(out, blob))
    gib = blob_len / (1 << 30)
    res = {"encode_gibs": round(gib / te, 3), "decode_gibs": round(gib / td, 3),
           "encode_decode_gibs": round(gib / (te + td), 3),
           "encode_ms": round(te * 1e3, 2), "decode_ms": round(td * 1e3, 2),
           "decode_roundtrip_ok": ok,
           "note": "rs2_encode_with_metadata + rs2_decode_blob on pageable host buffers "
                   f"(reused), best of {reps}; PCIe-inclusive, never `value`"}
    # the same calls with the caller's buffers registered once (rs2_host_register): the DMA
    # moves straight between them and the device, no staging ring
    bufs = [blob, prim, sec, out]
    t0 = time.perf_counter()
    for b in bufs:
        assert L.rs2_host_register(b.ctypes.data, b.nbytes) == 0, _lib.last_error()
    treg = time.perf_counter() - t0
    try:
        out[:] = 1
        te2, td2 = best(encode), best(decode)
        ok2 = bool(np.array_equal(out, blob))
    finally:
        for b in bufs:
            L.rs2_host_unregister(b.ctypes.data)
    res["registered"] = {"encode_gibs": round(gib / te2, 3), "decode_gibs": round(gib / td2, 3),
                         "encode_decode_gibs": round(gib / (te2 + td2), 3),
                         "encode_ms": round(te2 * 1e3, 2), "decode_ms": round(td2 * 1e3, 2),
                         "register_ms": round(treg * 1e3, 1), "decode_roundtrip_ok": ok2}
    return res


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_flags() -> list:
    """The SIMD features the CPU restatement could use (it is built for AVX2)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("flags"):
                have = set(line.split(":", 1)[1].split())
                return [f for f in ("avx2", "avx512f", "avx512bw", "gfni", "vpclmulqdq")
                        if f in have]
    except OSError:
        pass
    return []


def device_copy_gbs(dev, mib: int = 1024, reps: int = 10) -> float:
    """Measured device-to-device copy bandwidth (read + write bytes / s) of one large buffer:
    the practical HBM ceiling quoted beside the 8 TB/s spec peak."""
    import torch
    a = torch.empty(mib << 20, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize(dev)
    gbs = 2 * a.numel() * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return round(gbs, 1)


def cpu_share() -> tuple:
    """Host threads for the CPU twins: this GPU's share of the host.  The pool's boxes grant one
    GPU 16 CPUs and say so in OMP_NUM_THREADS (16 there, while os.cpu_count() shows the whole
    machine); without it, the visible CPUs / 8 GPUs of a full node.  Never more than this
    process may run on (sched_getaffinity).  Returns (threads, rule)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        share, rule = int(omp), f"OMP_NUM_THREADS={omp} (the box's CPU share of one GPU)"
    else:
        share = max(1, (os.cpu_count() or 8) // 8)
        rule = f"{os.cpu_count()} visible CPUs / 8 GPUs"
    threads = max(1, min(share, avail))
    return threads, f"{rule}; {avail} CPUs in this process's affinity -> {threads} threads"


def cpu_baseline(sample_mib: float, n: int, node: bool = True, node_recovers: int = 16,
                 c3_blobs: int = 128):
    """Time the CPU restatement of the reference path (oracle/rs2_cpu.c: reed-solomon-simd's
    AVX2 nibble-table FFT codec + Blake2b Merkle) on encode+decode of `sample_mib` blobs at the
    same n: one blob on one thread (the reference encodes a blob on one thread), and one blob per
    thread on this GPU's share of the host threads (cpu_share; the reference parallelises over
    blobs at its call sites, rayon in walrus-sdk/src/node_client.rs:3182).  `value` / `cores`
    are the multi-thread run.  Also C3's twin (BASELINE config C3: `c3_blobs` x 4 MiB, one blob
    per thread at a time, rs2_cpu_bench c3) and the storage-node side's.  Test infrastructure:
    measured beside the GPU, never part of the product path."""
    exe = os.path.join(ROOT, "oracle", "build", "rs2_cpu_bench")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=False,
                       capture_output=True)
    if not os.path.exists(exe):
        return {"value": None, "unit": "GiB/s", "cores": 1, "kind": "port",
                "sample": "oracle/build/rs2_cpu_bench missing (make -C oracle)"}
    threads, cores_rule = cpu_share()

    def run(t):
        res = subprocess.run([exe, str(n), str(int(sample_mib * (1 << 20))), str(t)],
                             capture_output=True, text=True, timeout=900)
        if res.returncode != 0:
            raise RuntimeError(f"rs2_cpu_bench failed (rc {res.returncode}): {res.stderr[-200:]}")
        return json.loads(res.stdout.strip().splitlines()[-1])

    try:
        one = run(1)
        many = run(threads) if threads > 1 else one
    except (RuntimeError, subprocess.TimeoutExpired) as e:
        return {"value": None, "unit": "GiB/s", "cores": threads, "kind": "port", "sample": str(e)}
    # the storage-node side's twin (bench.node_leg): the C port verifying every sliver of one
    # blob of the same size, serving n recovery symbols with proofs and recovering primary
    # slivers from K_s symbols, on the same host threads
    node_side = None
    if node:
        try:
            res = subprocess.run([exe, "node", str(n), str(int(sample_mib * (1 << 20))),
                                  str(threads), str(node_recovers)],
                                 capture_output=True, text=True, timeout=900)
            node_side = (json.loads(res.stdout.strip().splitlines()[-1]) if res.returncode == 0
                         else {"error": f"rc {res.returncode}: {res.stderr[-200:]}"})
        except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
            node_side = {"error": str(e)}
    c3 = None
    if c3_blobs:
        try:
            res = subprocess.run([exe, "c3", str(n), str(4 << 20), str(c3_blobs), str(threads)],
                                 capture_output=True, text=True, timeout=900)
            c3 = (json.loads(res.stdout.strip().splitlines()[-1]) if res.returncode == 0
                  else {"error": f"rc {res.returncode}: {res.stderr[-200:]}"})
        except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
            c3 = {"error": str(e)}
    return {"value": round(many["gibs"], 6), "unit": "GiB/s", "cores": many["cores"],
            "kind": "port", "sample": many["sample"] + f"; host CPU: {_cpu_model()}",
            "cores_rule": cores_rule, "c3_twin": c3,
            "host_cpus_visible": os.cpu_count(), "cpu_simd_flags": _cpu_flags(),
            "single_thread_gibs": round(one["gibs"], 6), "encode_s": one["encode_s"],
            "decode_s": one["decode_s"], "multi_thread_wall_s": many["wall_s"],
            "ok": bool(one["ok"] and many["ok"]), "node_side": node_side}


if __name__ == "__main__":
    main()
