"""Per-queue timeline of the SMT steps in a rocprofv3 kernel-trace CSV: how long the compute queue
sits idle inside a step (waits on the wgrad stream, host gaps) and how much of the wgrad stream's
work is still running after the compute queue's last backward kernel (the exposed tail that the
optimizer launch waits for). Steps are delimited by adamw_tiles_kernel as in scripts/trace_steps.py.

    python scripts/diag/stream_tail.py trace.csv [label]
"""
import collections
import csv
import json
import sys


def main(path, label=""):
    rows = list(csv.DictReader(open(path)))
    qkey = "Queue_Id"                              # Stream_Id is 0 without HIP API tracing
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw_tiles_kernel" in r["Kernel_Name"]]
    out = []
    for a, b in zip(idx[:-1], idx[1:]):
        seg = rows[a + 1:b + 1]
        t0 = int(seg[0]["Start_Timestamp"])
        opt = seg[-1]                                   # this step's adamw_tiles launch
        busy = collections.Counter()
        gemm = collections.Counter()
        for r in seg:
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            busy[r[qkey]] += d
            if r["Kernel_Name"].startswith(("Cijk", "Custom_Cijk")):
                gemm[r[qkey]] += d
        compute = max(gemm, key=gemm.get) if gemm else opt[qkey]
        # idle gaps on the compute queue (kernel end -> next kernel start on the same queue)
        cq = [r for r in seg if r[qkey] == compute]
        gaps = []
        for p, n in zip(cq[:-1], cq[1:]):
            g = int(n["Start_Timestamp"]) - int(p["End_Timestamp"])
            if g > 0:
                gaps.append((g, p["Kernel_Name"][:60], n["Kernel_Name"][:60]))
        gaps.sort(reverse=True)
        side = [r for r in seg if r[qkey] != compute]
        side_end = max((int(r["End_Timestamp"]) for r in side), default=t0)
        # the compute queue's last kernel before the optimizer
        pre = [r for r in cq if r is not opt]
        c_end = int(pre[-1]["End_Timestamp"]) if pre else t0
        out.append({
            "label": label,
            "wall_ms": round((int(opt["Start_Timestamp"]) - t0) / 1e6, 2),
            "compute_queue": compute,
            "compute_busy_ms": round(busy[compute] / 1e6, 2),
            "compute_idle_ms": round(sum(g for g, _, _ in gaps) / 1e6, 2),
            "largest_gaps_ms": [(round(g / 1e6, 3), p, n) for g, p, n in gaps[:5]],
            "side_busy_ms": round(sum(v for k, v in busy.items() if k != compute) / 1e6, 2),
            "side_kernels": len(side),
            "tail_after_compute_ms": round(max(0, side_end - c_end) / 1e6, 3),
            "optimizer_wait_ms": round((int(opt["Start_Timestamp"]) - c_end) / 1e6, 3),
        })
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:3])
