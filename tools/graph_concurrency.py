"""Do parallel branches of a captured HIP graph run concurrently? Two small-grid kernels (few workgroups, long
running) on forked streams vs the same two in sequence; eager and graph replay."""
import time

import torch


def work(x, n):
    for _ in range(n):
        x = torch.sin(x) * 1.0001
    return x


def main():
    dev = torch.device("cuda")
    a = torch.randn(64 * 256, device=dev)      # small: a handful of workgroups per launch
    b = torch.randn(64 * 256, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    n = 200

    def seq():
        work(a, n)
        work(b, n)

    def par():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            work(a, n)
        with torch.cuda.stream(s2):
            work(b, n)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    def timeit(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / reps * 1e3

    print(f"eager seq {timeit(seq):.2f} ms  eager par {timeit(par):.2f} ms", flush=True)
    for name, fn in (("seq", seq), ("par", par)):
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fn()
        torch.cuda.current_stream().wait_stream(side)
        with torch.cuda.graph(g):
            fn()
        print(f"graph {name} {timeit(g.replay):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
