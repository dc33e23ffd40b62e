"""Do two torch streams run concurrently on this box? A bf16 GEMM chain on one stream and an
HBM-bound copy chain on another, timed alone and together (HIP events on the default stream after
joining both). Together ~= max(alone) means they overlap; ~= sum means one hardware queue serialises
them. Prints one JSON line per stream configuration (default priority; side stream at priority -1)."""
import json
import time

import torch


def main():
    dev = torch.device("cuda")
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    c = torch.empty(8192, 8192, device=dev, dtype=torch.bfloat16)
    x = torch.empty(512 * 1024 * 1024, device=dev, dtype=torch.uint8)
    y = torch.empty_like(x)

    def gemms():
        for _ in range(20):
            torch.mm(a, b, out=c)

    def copies():
        for _ in range(40):
            y.copy_(x)

    def timed(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3

    for prio in (0, -1):
        s1 = torch.cuda.Stream(dev)
        s2 = torch.cuda.Stream(dev, priority=prio)

        def on(s, fn):
            def run():
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    fn()
                torch.cuda.current_stream().wait_stream(s)
            return run

        def both():
            s1.wait_stream(torch.cuda.current_stream())
            s2.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s1):
                gemms()
            with torch.cuda.stream(s2):
                copies()
            torch.cuda.current_stream().wait_stream(s1)
            torch.cuda.current_stream().wait_stream(s2)

        for _ in range(2):
            timed(on(s1, gemms)), timed(on(s2, copies)), timed(both)
        ga = min(timed(on(s1, gemms)) for _ in range(3))
        cb = min(timed(on(s2, copies)) for _ in range(3))
        tb = min(timed(both) for _ in range(3))
        print(json.dumps({"side_priority": prio, "gemm_ms": round(ga, 2), "copy_ms": round(cb, 2),
                          "together_ms": round(tb, 2), "sum_ms": round(ga + cb, 2),
                          "overlap_fraction": round((ga + cb - tb) / min(ga, cb), 3)}), flush=True)


if __name__ == "__main__":
    main()
