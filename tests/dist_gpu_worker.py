"""One rank of tests/test_gpu_dist.py (run under torch.distributed.run, every rank on cuda:0).

Partitioned encode_with_metadata (walrus_amd/partition.py: rows phase, all-to-all, columns
phase, all-to-all of leaf digests, row trees, all-to-all of primary-sliver symbols into
sliver-pair ownership, all-gather of the roots) and the decode of the
blob from K_p primary slivers that arrive on rank 0 (scatter of column ranges, column decodes,
gather), with the HIP engine (DeviceOps) and the exchanges over gloo through host memory
(HostStagedExchange).  Checked against the committed golden `c4s_n1000_24MiB` (C restatement,
tests/golden/make_fullsize.py) and the blob.  Rank 0 prints one `DIST_RESULT {json}` line.
Test infrastructure: the golden's generator is imported only for its PCG64 blob bytes.
"""
import base64
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import walrus_amd as W  # noqa: E402
from walrus_amd import partition as P  # noqa: E402
from make_fullsize import blob_bytes  # noqa: E402

CASE = "c4s_n1000_24MiB"


def main():
    backend = sys.argv[sys.argv.index("--backend") + 1] if "--backend" in sys.argv else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    with open(os.path.join(ROOT, "tests", "golden", "rs2_fullsize.json")) as f:
        case = [c for c in json.load(f)["cases"] if c["name"] == CASE][0]
    n, length = case["n_shards"], case["blob_len"]
    dev = torch.device("cuda", 0)
    host_blob = blob_bytes(case["seed"], length).copy()
    blob = torch.from_numpy(host_blob).to(dev)
    part = P.Partition.for_blob(n, length, world)
    # gloo: every collective staged through host memory (several ranks on the one GPU);
    # nccl: RCCL on the device buffers (one rank per GPU)
    ops = P.DeviceOps()
    ex = P.DistExchange() if backend == "nccl" else P.HostStagedExchange()
    res = {"rank": rank, "world": world, "backend": backend}

    # encode: every rank ends with all pair hashes and the BlobId
    enc = P.encode_distributed(part, P.rows_of_blob(part, blob, rank, dev), ops, ex, dev)
    torch.cuda.synchronize()
    hashes = bytes(enc.hashes.cpu().numpy())
    bid = base64.urlsafe_b64encode(bytes(enc.blob_id.cpu().numpy())).decode().rstrip("=")
    meta_ok = (hashlib.sha256(hashes).hexdigest() == case["pair_hashes_sha256"]
               and bid == case["blob_id"])
    flags = torch.tensor([int(meta_ok)], dtype=torch.int32,
                         device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    res["meta_ok_all_ranks"] = bool(flags.item())
    res["blob_id"] = bid

    # the sliver pairs every rank assembled (primary i, secondary n-1-i for i in its pairs),
    # gathered to rank 0 and checked against the golden's digests of all primary / secondary
    # slivers in index order
    nt, pl, sl = part.nt, part.ks * part.s, part.kp * part.s
    pad_p = torch.zeros(nt * pl, dtype=torch.uint8, device=dev)
    pad_s = torch.zeros(nt * sl, dtype=torch.uint8, device=dev)
    pad_p[:enc.primary.numel()].copy_(enc.primary)
    pad_s[:enc.secondary.numel()].copy_(enc.secondary)
    all_p, all_s = ex.gather(pad_p), ex.gather(pad_s)
    if rank == 0:
        hp, hs = hashlib.sha256(), hashlib.sha256()
        for g in range(world):
            hp.update(bytes(all_p[g * nt * pl:(g * nt + part.nv(g)) * pl].cpu().numpy()))
        for g in reversed(range(world)):   # rank g holds secondary slivers cstart(g).. ascending
            hs.update(bytes(all_s[g * nt * sl:(g * nt + part.nv(g)) * sl].cpu().numpy()))
        res["primary_slivers_ok"] = hp.hexdigest() == case["primary_all_sha256"]
        res["secondary_slivers_ok"] = hs.hexdigest() == case["secondary_all_sha256"]
    del all_p, all_s, pad_p, pad_s

    # decode from the primary slivers where the encode left them (all-to-all of the chosen
    # slivers' column ranges, column decodes, gather to rank 0)
    kp = part.kp
    idx = sorted(int(i) for i in np.random.default_rng(7).permutation(n)[:kp])
    got = P.decode_distributed(part, enc, idx, ops, ex, dev)
    if rank == 0:
        res["decode_from_held_slivers_ok"] = bool(torch.equal(got, blob))

    # decode from K_p full primary slivers received on rank 0 (here: the single-GPU plan's
    # encode of the same blob, itself checked against the golden)
    slivers = None
    if rank == 0:
        plan = W.DevicePlan(n, length)
        info = plan.info
        pl = info.primary_sliver_len
        prim = torch.zeros(n * pl + 256, dtype=torch.uint8, device=dev)
        sec = torch.zeros(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
        meta = torch.zeros(n * 64 + 32, dtype=torch.uint8, device=dev)
        plan.encode_async(blob.data_ptr(), prim.data_ptr(), sec.data_ptr(), meta.data_ptr(),
                          meta[n * 64:].data_ptr())
        plan.sync()
        pv = prim[:n * pl].view(n, pl)
        res["plan_primary_ok"] = (hashlib.sha256(bytes(pv.cpu().numpy())).hexdigest()
                                  == case["primary_all_sha256"])
        slivers = pv[torch.tensor(idx, device=dev)].contiguous().view(-1)
    got = P.decode_from_slivers(part, slivers, idx, ops, ex, dev)
    torch.cuda.synchronize()
    if rank == 0:
        res["decode_from_slivers_ok"] = bool(torch.equal(got, blob))
        print("DIST_RESULT " + json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
