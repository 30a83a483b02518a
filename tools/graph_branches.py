"""Do independent branches of a captured HIP graph run concurrently on this ROCm, and what does one
dependent launch cost inside a graph?  (Decides whether backward wgrad work can hide behind the
dgrad -> BatchNorm chain on a forked stream.)

    python tools/graph_branches.py
Prints one JSON line: serial / forked replay times of two spin kernels, and per-launch cost of a
chain of tiny kernels on one stream vs split over two streams.
"""
import json

import torch


def replay_ms(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def capture(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def main():
    cycles = 200000
    side = torch.cuda.Stream()
    x = torch.zeros(1024, device="cuda")

    def serial():
        torch.cuda._sleep(cycles)
        torch.cuda._sleep(cycles)

    def forked():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        torch.cuda._sleep(cycles)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cycles)
        cur.wait_stream(side)

    def one():
        torch.cuda._sleep(cycles)

    def chain(n):
        def f():
            for _ in range(n):
                x.add_(1.0)
        return f

    def chain2(n):
        def f():
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            y = torch.zeros(1024, device="cuda")
            for _ in range(n // 2):
                x.add_(1.0)
            with torch.cuda.stream(side):
                for _ in range(n // 2):
                    y.add_(1.0)
            cur.wait_stream(side)
        return f

    out = {"one_sleep_ms": replay_ms(capture(one)), "serial_2_sleep_ms": replay_ms(capture(serial)),
           "forked_2_sleep_ms": replay_ms(capture(forked))}
    for n in (1, 100, 200):
        out["chain%d_us_per_launch" % n] = replay_ms(capture(chain(n))) * 1e3 / n
    out["chain200_2streams_us_per_launch"] = replay_ms(capture(chain2(200))) * 1e3 / 200
    print(json.dumps(out))


if __name__ == "__main__":
    main()
