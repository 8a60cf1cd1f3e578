"""Per-stage HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/pmc_run.sh).

Dispatches of the engine's kernels are mapped onto bench.py's stage names by kernel name
(rs2_encode_shared[_pipe]_kernel alternates cols_sys / cols_rep within a step).  Traffic per launch follows
MI355X_MICROARCH.md (HBM section): FETCH_SIZE is reported in KiB and counts half the bytes of
wide streaming reads on gfx950, so bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
usage: python tools/pmc_traffic.py gpurun_out/pmc profiles/pmc_traffic.json
"""
import collections
import csv
import glob
import json
import sys

SHARED = ["enc_cols_sys_codec", "enc_cols_rep_codec"]
SINGLE = {"rs2_encode_mixed": "enc_rows_codec", "rs2_decode_kernel": "dec_codec",
          "leaf_hash_kernel": "enc_leaf_hash", "merkle_trees_kernel": "enc_merkle_trees",
          "merkle_root_kernel": "enc_merkle_root", "build_mul_tables_kernel": "dec_setup",
          "symbol_copy_kernel": "symbol_copy"}


def load(root, counter):
    per = {}
    for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            d = int(r["Dispatch_Id"])
            name = r["Kernel_Name"]
            v = per.setdefault(d, [name, 0.0])
            v[1] += float(r["Counter_Value"])
    return per


def stages(per):
    out = collections.defaultdict(list)
    n_shared = n_leaf = 0
    # split leaf hashing (rs2_engine.cpp encode_device): two leaf dispatches per encode, the
    # primary slivers' run A on the side stream first
    n_dec = sum(1 for name, _ in per.values() if "rs2_decode_kernel" in name)
    leaf_split = n_dec > 0 and sum(1 for name, _ in per.values()
                                   if "leaf_hash_kernel" in name) == 2 * n_dec
    for d in sorted(per):
        name, val = per[d]
        if "rs2_encode_shared" in name:
            out[SHARED[n_shared % 2]].append(val)
            n_shared += 1
        elif "leaf_hash_kernel" in name and leaf_split:
            out[["enc_leaf_hash_a", "enc_leaf_hash"][n_leaf % 2]].append(val)
            n_leaf += 1
        else:
            for k, st in SINGLE.items():
                if k in name:
                    out[st].append(val)
    return out


# stages that are more than one dispatch per step (bench.py MULTI_LAUNCH: the row codec runs
# over the blob's whole rows, then its padded tail rows); their figures are per step
PER_STEP = {"enc_rows_codec": 2}


def mean(st, v):
    k = PER_STEP.get(st, 1)
    return sum(v) / (len(v) / k) if v else None


def main():
    root, dst = sys.argv[1], sys.argv[2]
    fetch = stages(load(root, "FETCH_SIZE"))
    write = stages(load(root, "WRITE_SIZE"))
    valu = stages(load(root, "SQ_INSTS_VALU"))
    lds = stages(load(root, "SQ_INSTS_LDS"))
    res = {}
    for st in sorted(set(fetch) | set(write)):
        f = fetch.get(st, [])
        w = write.get(st, [])
        fb = 2 * 1024 * mean(st, f) if f else None
        wb = 1024 * mean(st, w) if w else None
        vi = mean(st, valu.get(st, []))
        li = mean(st, lds.get(st, []))
        res[st] = {"hbm_bytes_per_launch": round((fb or 0) + (wb or 0)),
                   "read_bytes_per_launch": round(fb) if fb is not None else None,
                   "write_bytes_per_launch": round(wb) if wb is not None else None,
                   "valu_insts_per_launch": round(vi) if vi is not None else None,
                   "lds_insts_per_launch": round(li) if li is not None else None,
                   "launches": max(len(f), len(w)) // PER_STEP.get(st, 1)}
    res["_method"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU + SQ_INSTS_LDS in separate passes "
                      "of bench.py --steps 2 --warmup 1 --overlap off; bytes = 2*FETCH_SIZE*1024 + "
                      "WRITE_SIZE*1024 (gfx950 FETCH_SIZE counts half of wide streaming reads); "
                      "VALU / LDS = wave instructions; enc_rows_codec is per step (2 dispatches)")
    json.dump(res, open(dst, "w"), indent=1)
    for k, v in res.items():
        print(k, v)


if __name__ == "__main__":
    main()
