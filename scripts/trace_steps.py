"""Per-category kernel time of the SMT steps from a rocprofv3 kernel-trace CSV.

SMT steps are delimited by adamw_tiles_kernel dispatches (one per step): the region between two
consecutive ones is one step. Prints per-step wall (first start .. last end) and kernel-time by category.
``python scripts/trace_steps.py trace.csv adamw_multi_kernel``: the full fine-tuning warm-up steps
instead (one dense multi-tensor AdamW launch per parameter group and step: the first of each step's
burst delimits)."""
import collections
import csv
import sys


def cat(name):
    n = name
    if "wgrad_" in n or "colblock_gather" in n:
        return "smt_wgrad"
    if "grad_accumulate" in n or "block_score" in n:
        return "smt_harvest"
    if "adamw_multi" in n:
        return "dense_adamw"
    if "adamw" in n or "sq_norm" in n or "tile_copy" in n or "tile_scatter_t" in n:
        return "smt_optimizer"
    if "ce_fwd_kernel" in n or "ce_bwd_kernel" in n:
        return "loss(smt_ce)"
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        return "gemm(hipBLASLt)"
    if "attn_fwd_kernel" in n or "attn_dq_kernel" in n or "attn_dkdv_kernel" in n or "attn_delta_kernel" in n:
        return "attention(smt_flash)"
    if any(k in n for k in ("rmsnorm", "rope_kernel", "swiglu")):
        return "fused_llama_ops"
    if "attn_fwd" in n or "bwd_kernel" in n or "bwd_preprocess" in n:
        return "attention(aotriton)"
    if "SoftMax" in n or "nll_loss" in n or "log_softmax" in n:
        return "loss"
    if "reduce_kernel" in n:
        return "reductions"
    if "elementwise" in n or "Copy" in n or "copy" in n or "Cat" in n:
        return "elementwise"
    return "other"


def main(path, delim="adamw_tiles_kernel"):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if delim in r["Kernel_Name"]]
    # a burst of delimiter launches (one per parameter group) counts once: keep the last of each
    idx = [i for k, i in enumerate(idx) if k + 1 == len(idx) or idx[k + 1] - i > 8]
    if len(idx) < 2:
        print("need >= 2 SMT steps")
        return
    for a, b in zip(idx[:-1], idx[1:]):
        seg = rows[a + 1:b + 1]
        wall = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
        by = collections.Counter()
        cnt = collections.Counter()
        for r in seg:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            by[cat(r["Kernel_Name"])] += d
            cnt[cat(r["Kernel_Name"])] += 1
        busy = sum(by.values())
        print(f"step: wall {wall:.1f} ms, kernel-busy {busy:.1f} ms, dispatches {len(seg)}")
        for k, v in by.most_common():
            print(f"   {k:22s} {v:8.1f} ms  {100 * v / wall:5.1f}%  n={cnt[k]}")
    # the last step's non-GEMM kernels by name
    seg = rows[idx[-2] + 1:idx[-1] + 1]
    per = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        n = r["Kernel_Name"]
        if cat(n) == "gemm(hipBLASLt)":
            continue
        per[n][0] += 1
        per[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print("last step, non-GEMM kernels:")
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"   {t:8.2f} ms  n={c:4d}  {n[:140]}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
