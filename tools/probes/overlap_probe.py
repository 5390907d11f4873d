"""Does a persistent kernel that holds only part of the chip (the encoder BiLSTM: one workgroup
per (direction, utterance), 64 workgroups at B=32) overlap with an independent weight-gradient
GEMM (256 x 1024 x 16000, the decoder LSTM's dW shape) when both are branches of ONE hipGraph?

Prints: BiLSTM alone, GEMM alone, both serial in one graph, both as parallel branches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
B, N, U = 32, 200, 128
f32 = dict(device=dev, dtype=torch.float32)
X = torch.randn(B, N, 4 * U, **f32) * 0.1
W = torch.randn(U, U, 4, **f32) * 0.05
lengths = torch.full((B,), N, dtype=torch.int64, device=dev)
H = torch.empty(B, N, 2 * U, **f32)
hist = [torch.zeros(N + 1, B, U, **f32) for _ in range(4)]
G = [torch.empty(N, B, 4 * U, **f32) for _ in range(2)]
A = torch.randn(16000, 256, **f32)
Bm = torch.randn(16000, 1024, **f32)
C = torch.empty(256, 1024, **f32)


def lstm():
    K.encoder_lstm_fwd(B=B, N=N, U=U, zc=0.1, zh=0.1, X_fw=X, X_bw=X, x_sb=X.stride(0),
                       x_sn=X.stride(1), W_fw=W, W_bw=W, mc_fw=None, mh_fw=None, mc_bw=None,
                       mh_bw=None, lengths=lengths, H=H, h_sb=H.stride(0), h_sn=H.stride(1),
                       CS_fw=hist[0], HS_fw=hist[1], CS_bw=hist[2], HS_bw=hist[3], G_fw=G[0],
                       G_bw=G[1])


def gemm():
    for _ in range(3):
        K.gemm(A.t(), Bm, C)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
for s in (sa, sb):
    with torch.cuda.stream(s):
        K._gemm_ws(dev)
        lstm()
        gemm()
torch.cuda.synchronize()


def capture(fn):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        K._gemm_ws(dev)
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    return g


g_l = capture(lstm)
g_g = capture(gemm)
g_ser = capture(lambda: (lstm(), gemm()))


def par():
    main = torch.cuda.current_stream()
    sa.wait_stream(main)
    sb.wait_stream(main)
    with torch.cuda.stream(sa):
        lstm()
    with torch.cuda.stream(sb):
        gemm()
    main.wait_stream(sa)
    main.wait_stream(sb)


g_par = capture(par)
tl, tg, ts, tp = timed(g_l.replay), timed(g_g.replay), timed(g_ser.replay), timed(g_par.replay)
print(f"BiLSTM alone {tl:.1f} us; 3 GEMMs alone {tg:.1f} us; serial graph {ts:.1f} us; "
      f"parallel branches {tp:.1f} us (perfect overlap would be {max(tl, tg):.1f})", flush=True)
# eager two streams
tpe = timed(par)
print(f"eager two streams {tpe:.1f} us", flush=True)
