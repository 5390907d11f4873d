"""Do independent kernel chains overlap on MI355X?  (graph branches vs graphs on streams)"""
import torch

dev = torch.device("cuda:0")
N = 300


def chain(x):
    for _ in range(N):
        x.mul_(1.0001)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for numel in (1 << 12, 1 << 20):
    a = torch.ones(numel, device=dev)
    b = torch.ones(numel, device=dev)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        chain(a)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        main = torch.cuda.current_stream()
        sa.wait_stream(main)
        sb.wait_stream(main)
        with torch.cuda.stream(sa):
            chain(a)
        with torch.cuda.stream(sb):
            chain(b)
        main.wait_stream(sa)
        main.wait_stream(sb)
    gA = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gA):
        chain(a)
    gB = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gB):
        chain(b)

    def two_graphs():
        main = torch.cuda.current_stream()
        sa.wait_stream(main)
        sb.wait_stream(main)
        with torch.cuda.stream(sa):
            gA.replay()
        with torch.cuda.stream(sb):
            gB.replay()
        main.wait_stream(sa)
        main.wait_stream(sb)

    t1 = timed(g1.replay)
    t2 = timed(g2.replay)
    t3 = timed(two_graphs)
    print(f"numel {numel}: one chain {t1 * 1e3 / N:.2f} us/kernel; two chains in one graph "
          f"{t2 * 1e3 / N:.2f} us per pair; two graphs on two streams {t3 * 1e3 / N:.2f} us per pair",
          flush=True)
