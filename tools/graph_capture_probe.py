"""Probe multi-stream hipGraph capture patterns (each mode in its own process).

    python tools/graph_capture_probe.py            # runs every mode as a child process
    python tools/graph_capture_probe.py <mode>     # one mode
"""
import subprocess
import sys

import torch

MODES = ["torch_ops_2chunks", "torch_ops_refork", "model_seq", "model_chunk4", "lib_gemm_side"]


def torch_ops(nchunks, keep, refork=False):
    dev = torch.device("cuda:0")
    side = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
    x = torch.ones(1 << 16, device=dev)
    y = torch.zeros_like(x)
    z = torch.zeros_like(x)
    kept = []

    def handoff(src, dst):
        ev = torch.cuda.Event()
        ev.record(src)
        dst.wait_event(ev)
        if keep:
            kept.append(ev)

    def body():
        main = torch.cuda.current_stream()
        for s in side:
            s.wait_stream(main)
        for _ in range(nchunks):
            x.add_(1.0)
            handoff(main, side[0])
            with torch.cuda.stream(side[0]):
                y.add_(x)
            handoff(side[0], side[1])
            with torch.cuda.stream(side[1]):
                z.add_(y)
        for s in side:
            main.wait_stream(s)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
        if refork:       # same side streams forked/joined a second time in one capture
            body()
    g.replay()
    torch.cuda.synchronize()
    print("ok", float(z[0]))


def lib_gemm_side():
    """one libsat GEMM on a side stream inside a capture"""
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import _sat_path
    _sat_path.load()
    from sat_amd import kernels as K
    dev = torch.device("cuda:0")
    side = torch.cuda.Stream(dev)
    a = torch.randn(64, 64, device=dev)
    c = torch.zeros(64, 64, device=dev)

    def body():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            K.gemm(a, a, c)
        torch.cuda.current_stream().wait_stream(side)

    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    g.replay()
    torch.cuda.synchronize()
    print("ok")


def model(chunk, fwd_pipe=True, bwd_pipe=True, fwd_only=False):
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import _sat_path
    _sat_path.load()
    from sat_amd import data, engine, hparams, train
    hp = hparams.ljspeech_hparams()
    from sat_amd import pipeline, backward, model as MD
    m = engine.Tacotron(hp, "cuda", seed=1, pipeline_chunk=chunk)
    b = data.synthetic_batch(hp, 3, N=19, T=30, shape="ljs", seed=8)
    batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
    if fwd_only:
        def body():
            return m.forward(batch, None, training=False, need_grad=False)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body()
        g.replay()
        torch.cuda.synchronize()
        print("ok fwd only")
        return
    pipe = m.pipe
    if not fwd_pipe or not bwd_pipe:
        seq = pipeline.SEQUENTIAL
        orig_f, orig_b = m.forward, m.backward

        def fwd(batch, masks=None, training=True, need_grad=True):
            return MD.model_forward(m.P, m.bn, m.hp, m.d, batch, masks, training, m.ws,
                                    compute_grad_seeds=need_grad, attn_tile=m.attn_tile,
                                    pipe=pipe if fwd_pipe else seq)

        def bwd(saved, zero=True):
            if zero:
                m.grads.zero_()
            backward.model_backward(m.P, m.G, m.hp, m.d, saved, m.ws, attn_tile=m.attn_tile,
                                    pipe=pipe if bwd_pipe else seq)
        m.forward, m.backward = fwd, bwd
    tr = train.Trainer(m, 3, batch["source"].shape[1], batch["mel"].shape[1] // 2, seed=5)
    g = train.GraphedStep(tr, batch, warmup=1)
    g.replay()
    torch.cuda.synchronize()
    print("ok", float(tr.last_loss.item()))


def run(mode):
    if mode == "torch_ops_2chunks":
        torch_ops(2, False)
    elif mode == "torch_ops_8chunks":
        torch_ops(8, False)
    elif mode == "torch_ops_keep_events":
        torch_ops(8, True)
    elif mode == "torch_ops_refork":
        torch_ops(3, False, refork=True)
    elif mode == "model_seq":
        model(0)
    elif mode == "model_fwd_only_capture":
        model(4, fwd_only=True)
    elif mode == "model_fwd_pipe_bwd_seq":
        model(4, bwd_pipe=False)
    elif mode == "model_fwd_seq_bwd_pipe":
        model(4, fwd_pipe=False)
    elif mode == "model_chunk4":
        model(4)
    elif mode == "lib_gemm_side":
        lib_gemm_side()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        for mode in MODES:
            r = subprocess.run([sys.executable, __file__, mode], capture_output=True, text=True,
                               timeout=300)
            tail = [l for l in (r.stdout + r.stderr).strip().splitlines()
                    if "amdgpu.ids" not in l][-2:]
            print(f"{mode:24s} rc={r.returncode} {tail}", flush=True)
