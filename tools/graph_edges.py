"""Micro-benchmark of HIP-graph stream fork/join cost (captured torch graphs):
per-iteration time of a chain A -> {main branch || side branch} -> join,
with torch.cuda._sleep kernels (~21.6 us per unit) as the work.  Shows
which branch pays the cross-queue dependency latency."""
import torch

torch.cuda.set_device(0)
U = 50000  # _sleep cycles per unit (~21.6 us)


def make(main_units, side_units, side_first, side):
    def body():
        for _ in range(20):
            torch.cuda._sleep(U)  # A
            if side_units is None:
                for u in main_units:
                    torch.cuda._sleep(u)
                continue
            side.wait_stream(torch.cuda.current_stream())  # fork

            def s_work():
                with torch.cuda.stream(side):
                    for u in side_units:
                        torch.cuda._sleep(u)

            if side_first:
                s_work()
            for u in main_units:
                torch.cuda._sleep(u)
            if not side_first:
                s_work()
            torch.cuda.current_stream().wait_stream(side)  # join
    return body


def bench(main_units, side_units, side_first=False):
    side = torch.cuda.Stream()
    body = make(main_units, side_units, side_first, side)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / 200 * 1e3


cases = [
    ("serial A+2U", [U, U], None, False),
    ("main 2U | side 0.1U", [U, U], [U // 10], False),
    ("main 0.1U | side 2U", [U // 10], [U, U], False),
    ("main 2U | side 0.1U, side captured first", [U, U], [U // 10], True),
    ("main 0.1U | side 2U, side captured first", [U // 10], [U, U], True),
    ("main 2U | side 2U", [U, U], [U, U], False),
    ("main 2x(U) | side 1x(2U)", [U, U], [2 * U], False),
    ("main 1x(2U) | side 2x(U)", [2 * U], [U, U], False),
]
for name, m, sd, sf in cases:
    print(f"{name:45s} {bench(m, sd, sf):8.2f} us/iter", flush=True)
