"""Drive the persistent decoder attention kernels (dec_attn_fwd8 / bwd8) in the training
configuration of the bench (B=32, N=200, T=1000, zoneout masks, energy-tanh history kept) for
rocprofv3 PMC passes, one counter group per run:

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o pmc -- \
        python3 tools/pmc_persistent.py
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o pmc -- \
        python3 tools/pmc_persistent.py
    python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write dec_attn_fwd_kernel \
        > profiles/rNN_dec_attn_fwd_pmc.json
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import data, engine, hparams  # noqa: E402


def main(B=32, N=200, T=1000, passes=3):
    hp = hparams.ljspeech_hparams()
    m = engine.Tacotron(hp, "cuda", seed=1234)
    b = data.synthetic_batch(hp, B, N=N, T=T, shape="max", seed=1)
    batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
    mk = {k: torch.tensor(v).cuda()
          for k, v in data.synthetic_masks(hp, B, N, T // hp.outputs_per_step, seed=2).items()}
    for _ in range(passes):
        out, sv = m.forward(batch, mk, training=True)
        m.backward(sv)               # the BPTT kernel (dec_attn_bwd8_kernel) too
        del out, sv
    torch.cuda.synchronize()
    print("forward + backward passes", passes)


if __name__ == "__main__":
    main()
