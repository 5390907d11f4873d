#!/usr/bin/env python3
"""Teacher-forced training throughput of the MI355X Self-attention Tacotron (BASELINE.json).

metric : teacher-forced mel frames/sec, LJSpeech batch=32, 1/2/4/8 MI355X
step   : one full training step -- dropout/zoneout mask draw, forward (encoder, 500-step decoder
         loop, causal self-attention head, loss), hand-written BPTT, RCCL gradient all-reduce
         (N>1), global-norm clip + Adam -- on a synthetic LJSpeech-shaped batch resident in HBM
         (B=32 per GPU, 200 chars, 1000 mel frames x 80 bins, r=2; random text, random mel,
         random-init weights of the LJSpeech self-attention-tacotron.json architecture).
value  : whole-job frames/s = n_gpus * B * T * steps / max-over-ranks wall time (weak scaling).

Run:  python bench.py [--gpus N --steps K --warmup W]
      torchrun --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
Extra objects on the JSON line: ``roofline`` (the dual-source attention tile kernel, timed live
with HIP events on the stream it runs on) and ``cpu_baseline`` (the CPU oracle, bounded sample).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import _sat_path  # noqa: E402

_sat_path.load()

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "teacher-forced mel frames/sec, LJSpeech batch=32, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--chars", type=int, default=200)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true",
                    help="skip the attention-kernel probe (profiling runs of the step alone)")
    ap.add_argument("--cpu-baseline-batch", type=int, default=2)
    ap.add_argument("--cpu-baseline-steps", type=int, default=4)
    ap.add_argument("--attn-tile", type=int, default=32)
    ap.add_argument("--pipeline-chunk", type=int, default=40,
                    help="decoder steps per chunk of the multi-stream recurrence pipeline (0 = off)")
    return ap.parse_args()


def attention_probe(trainer, hp, d, B, N, tile):
    """Average duration of the dual-source attention tile kernel over all decoder steps of the
    last training step's state, timed with HIP events on the launching stream, and its
    algorithmic bytes per launch."""
    from sat_amd import kernels as K
    sv = trainer.last_saved["dec"].tensors
    P = trainer.m.P
    Tp = sv["Q"].shape[0]
    ntiles = (N + tile - 1) // tile
    pst = K.part_stride(d.m1, d.m2)
    e1 = torch.empty(B, N, device="cuda")
    e2 = torch.empty(B, N, device="cuda")
    part = torch.empty(B, ntiles, pst, device="cuda")
    dummy = torch.empty(B, N, device="cuda")
    ctx = torch.empty(B, d.m1 + d.m2, device="cuda")
    a1 = "decoder/attention1"

    def launch(t):
        K.attn_step_fwd(
            B=B, N=N, D1=d.d1, M1=d.m1, D2=d.d2, M2=d.m2, F=d.loc_f, KW=d.loc_k, NT=tile,
            ntiles=ntiles, att1_forward=1, u=0.5, q=sv["Q"][t], q_sb=d.d1 + d.d2,
            K1=sv["K1"], V1=sv["V1"], K2=sv["K2"], V2=sv["V2"],
            lengths=trainer.batch_lengths, s_prev=sv["S1"][t], a_prev=sv["AL1"][t],
            v1=P[f"{a1}/attention_variable"], b1=P[f"{a1}/attention_bias"],
            convW=P[f"{a1}/location_conv/kernel"], convb=P[f"{a1}/location_conv/bias"],
            locW=P[f"{a1}/location_layer/kernel"], v2=P["decoder/attention2/attention_v"],
            e1=e1, e2=e2, part=part, part_stride=pst, s_out=dummy, a_out=dummy,
            s2_out=dummy, ctx=ctx, ctx_sb=d.m1 + d.m2, stats=None, phases=1)

    for t in range(min(Tp, 20)):
        launch(t)
    torch.cuda.synchronize()
    # capture the T' launches of one decoder pass so host launch cost is out of the timing
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for t in range(Tp):
            launch(t)
    graph.replay()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 4
    ev0.record()
    for _ in range(reps):
        graph.replay()
    ev1.record()
    torch.cuda.synchronize()
    avg_s = ev0.elapsed_time(ev1) / 1e3 / (reps * Tp)
    f = 4  # fp32
    bytes_launch = f * (
        B * N * (d.d1 + d.m1 + d.d2 + d.m2)        # K1, V1, K2, V2 streamed
        + 2 * B * N                                # s_{t-1}, alpha_{t-1}
        + B * (d.d1 + d.d2)                        # processed queries
        + 2 * B * N                                # e1, e2 written
        + B * ntiles * pst                         # partial records written
        + 2 * d.d1 + d.loc_f * d.d1 + d.loc_k * d.loc_f + d.loc_f + d.d2)   # weights
    achieved = bytes_launch / avg_s / 1e9
    traffic, pmc_src = _pmc_traffic()
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": "attn_energy_wide_kernel<5,16> (sat_attn_step_fwd tile phase)",
            "bytes_per_launch": int(bytes_launch), "avg_launch_us": round(avg_s * 1e6, 3),
            "launches_timed": reps * Tp,
            "note": "avg = HIP-event time of hipGraph-replayed back-to-back launches / count "
                    "(includes the ~1.5 us inter-kernel boundary); traffic = memory-side bytes "
                    "per launch from rocprofv3 FETCH_SIZE (x2, gfx950) + WRITE_SIZE passes "
                    f"({pmc_src}); L2 does not survive the kernel boundary, so K1/V1 are "
                    "re-fetched every decoder step"}


def _pmc_traffic():
    """Per-launch HBM bytes of the tile kernel from the newest committed PMC summary
    (profiles/rNN_attn_energy_pmc.json, made by tools/pmc_attention.py + tools/pmc_summary.py)."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                          "r*_attn_energy_pmc.json")))
    if not files:
        return None, "no PMC summary"
    try:
        d = json.load(open(files[-1]))
        return int(d["hbm_bytes_per_launch"]), os.path.basename(files[-1])
    except (OSError, ValueError, KeyError):
        return None, "unreadable PMC summary"


def cpu_baseline(hp, args):
    """The CPU oracle (float32 PyTorch-CPU restatement, test infrastructure) timed on this box's
    host cores on a bounded sample of the same workload: C1 = LJSpeech B=2 x (200 chars,
    1000 frames), one full training step (forward + autograd BPTT + Adam)."""
    from oracle import sat_oracle as O
    from sat_amd import data, params
    B = args.cpu_baseline_batch
    # the box's OMP_NUM_THREADS share (16 there); the affinity mask can list the whole machine
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0"))
                          or min(16, len(os.sched_getaffinity(0))))
    vals = params.init_params(hp, seed=1234)
    p = {k: v.requires_grad_(True) for k, v in O.to_torch(vals, torch.float32).items()}
    bufs = O.to_torch(params.init_bn_buffers(hp), torch.float32)
    batch = O.to_torch(data.synthetic_batch(hp, B, N=args.chars, T=args.frames, seed=7),
                       torch.float32)
    Tp = args.frames // hp.outputs_per_step
    masks = O.to_torch(data.synthetic_masks(hp, B, args.chars, Tp, seed=8), torch.float32)
    m = {k: torch.zeros_like(v) for k, v in p.items()}
    v2 = {k: torch.zeros_like(v) for k, v in p.items()}
    t0 = time.perf_counter()
    for s in range(args.cpu_baseline_steps):
        for q in p.values():
            q.grad = None
        out = O.model_forward(p, bufs, hp, batch, masks, training=True)
        out["loss"].backward()
        with torch.no_grad():
            grads, _ = O.clip_by_global_norm([q.grad for q in p.values()], 1.0)
            lr = O.learning_rate(hp.initial_learning_rate, s)
            for (k, q), g in zip(p.items(), grads):
                new, m[k], v2[k] = O.adam_tf(q, g, m[k], v2[k], lr, s + 1)
                q.copy_(new)
    dt = (time.perf_counter() - t0) / args.cpu_baseline_steps
    return {"value": round(B * args.frames / dt, 2), "unit": "frames/s",
            "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"CPU oracle (float32 PyTorch-CPU restatement, not TF1.x), LJSpeech B={B} x "
                      f"{args.chars} chars x {args.frames} frames, {args.cpu_baseline_steps} "
                      f"full training step(s) (fwd + BPTT + Adam), {dt:.2f} s/step"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run")
    torch.cuda.set_device(local)
    dist = world > 1
    if dist:
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    from sat_amd import data, dp, engine, hparams, train
    hp = hparams.ljspeech_hparams()
    B, N, T = args.batch, args.chars, args.frames
    model = engine.Tacotron(hp, "cuda", seed=1234, attn_tile=args.attn_tile,
                            pipeline_chunk=args.pipeline_chunk)
    dp.broadcast_params(model.params)   # identical initial weights on every replica
    b = data.synthetic_batch(hp, B, N=N, T=T, shape="max", seed=1000 + rank * 1_000_000)
    batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
    trainer = train.Trainer(model, B, N, T // hp.outputs_per_step, seed=1234 + rank)
    trainer.batch_lengths = batch["source_length"]
    if args.no_graph:
        for _ in range(max(1, args.warmup)):
            trainer.step(batch)
        run = lambda: trainer.step(batch)  # noqa: E731
    else:
        g = train.GraphedStep(trainer, batch, warmup=1)
        for _ in range(args.warmup):
            g.replay()
        run = g.replay
    torch.cuda.synchronize()
    loss0 = float(trainer.last_loss.item())
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    dt = dp.max_over_ranks(dt, "cuda")
    loss1 = float(trainer.last_loss.item())
    frames = world * B * T * args.steps
    value = frames / dt
    roof = None if args.no_roofline else attention_probe(trainer, hp, model.d, B, N,
                                                         args.attn_tile)
    if rank == 0:
        cpu = None if args.no_cpu_baseline else cpu_baseline(hp, args)
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (random text ids 1..70, N(0,1) normalised mel, random-init weights)",
            "config": {"workload": "LJSpeech self-attention-tacotron.json teacher-forced training "
                                   "step (fwd + BPTT + Adam), configs[1]",
                       "global_batch": B * world, "per_gpu_batch": B, "chars": N,
                       "mel_frames": T, "num_mels": hp.num_mels, "r": hp.outputs_per_step,
                       "decoder_steps": T // hp.outputs_per_step, "parallelism": f"dp{world}",
                       "hip_graph": not args.no_graph, "params": model.num_params},
            "roofline": roof, "cpu_baseline": cpu,
            "loss_first_timed": round(loss0, 5), "loss_last": round(loss1, 5),
        }
        print(json.dumps(line), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
