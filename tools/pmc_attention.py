"""Drive the dual-source attention tile kernel alone (eager launches over one decoder pass of
real state) for rocprofv3 PMC passes:

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o pmc -- \
        python3 tools/pmc_attention.py
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o pmc -- \
        python3 tools/pmc_attention.py
    python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/...json
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import data, engine, hparams, train  # noqa: E402
from sat_amd import kernels as K  # noqa: E402


def main(B=32, N=200, T=1000, launches=200):
    hp = hparams.ljspeech_hparams()
    m = engine.Tacotron(hp, "cuda", pipeline_chunk=0)
    d = m.d
    b = data.synthetic_batch(hp, B, N=N, T=T, shape="max", seed=1)
    batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
    tr = train.Trainer(m, B, N, T // 2)
    with torch.no_grad():
        _, sv = m.forward(batch, None, training=False, need_grad=False)
    torch.cuda.synchronize()
    S = sv["dec"].tensors
    P = m.P
    ntiles = (N + 31) // 32
    pst = K.part_stride(d.m1, d.m2)
    f = dict(device="cuda")
    E1, E2 = torch.empty(B, N, **f), torch.empty(B, N, **f)
    PART = torch.empty(B, ntiles, pst, **f)
    dummy = torch.empty(B, N, **f)
    ctx = torch.empty(B, d.m1 + d.m2, **f)
    a1 = "decoder/attention1"
    Tp = S["Q"].shape[0]
    for i in range(launches):
        t = i % Tp
        K.attn_step_fwd(
            B=B, N=N, D1=d.d1, M1=d.m1, D2=d.d2, M2=d.m2, F=d.loc_f, KW=d.loc_k, NT=32,
            ntiles=ntiles, att1_forward=1, u=0.5, q=S["Q"][t], q_sb=d.d1 + d.d2, K1=S["K1"],
            V1=S["V1"], K2=S["K2"], V2=S["V2"], lengths=batch["source_length"],
            s_prev=S["S1"][t], a_prev=S["AL1"][t], v1=P[f"{a1}/attention_variable"],
            b1=P[f"{a1}/attention_bias"], convW=P[f"{a1}/location_conv/kernel"],
            convb=P[f"{a1}/location_conv/bias"], locW=P[f"{a1}/location_layer/kernel"],
            v2=P["decoder/attention2/attention_v"], e1=E1, e2=E2, part=PART, part_stride=pst,
            s_out=dummy, a_out=dummy, s2_out=dummy, ctx=ctx, ctx_sb=d.m1 + d.m2, stats=None,
            phases=1)
    torch.cuda.synchronize()
    print("launched", launches)


if __name__ == "__main__":
    main()
