"""Do the independent branches of a captured hipGraph run concurrently on this stack?

Two chains of small (GPU-underfilling) kernels, A and B, each N launches long:
serial (one stream), eager two streams, and both variants captured into a graph.  If the
graph's two-stream time is near max(A, B) rather than A + B, the branches overlap - the
condition for moving ResNet's weight-gradient kernels onto a side stream.
"""
import torch


def chain(x, n):
    for _ in range(n):
        x = torch.tanh(x @ x) * 0.5
    return x


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def main():
    dev = torch.device("cuda")
    n = 50
    a = torch.randn(128, 128, device=dev) * 0.05
    b = torch.randn(128, 128, device=dev) * 0.05
    side = torch.cuda.Stream()

    def serial():
        chain(a, n)
        chain(b, n)

    def two():
        main_s = torch.cuda.current_stream()
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            chain(b, n)
        chain(a, n)
        main_s.wait_stream(side)

    res = {"one_chain_us": timed(lambda: chain(a, n)), "serial_us": timed(serial), "two_streams_us": timed(two)}
    for name, fn in (("graph_serial_us", serial), ("graph_two_streams_us", two)):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            fn()
        res[name] = timed(g.replay)
    print(res)


if __name__ == "__main__":
    main()
