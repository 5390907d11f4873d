#!/usr/bin/env python3
"""Teacher-forced training throughput of the MI355X Self-attention Tacotron (BASELINE.json).

metric : teacher-forced mel frames/sec, LJSpeech batch=32, 1/2/4/8 MI355X
step   : one full training step -- dropout/zoneout mask draw, forward (encoder, 500-step decoder
         loop, causal self-attention head, loss), hand-written BPTT, RCCL gradient all-reduce
         (N>1), global-norm clip + Adam -- on a synthetic LJSpeech-shaped batch resident in HBM
         (B=32 per GPU, 200 chars, 1000 mel frames x 80 bins, r=2; random text, random mel,
         random-init weights of the LJSpeech self-attention-tacotron.json architecture).
value  : whole-job frames/s = n_gpus * B * T * steps / max-over-ranks wall time (weak scaling).

Run:  python bench.py [--gpus N --steps K --warmup W]   (N > 1: starts N ranks itself)
      torchrun --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
Extra objects on the JSON line: ``roofline`` (the persistent decoder attention kernel, the
step's dominant kernel, timed live with HIP events on the stream it runs on), ``cpu_baseline``
(the CPU oracle, bounded sample), ``median_ms_per_step`` (per-step HIP events) and, at N=1, the
other single-GPU configs: ``c4_vctk_training`` (configs[3]) and ``c5_free_running``
(configs[4]).  Any training step skipped by the health guard aborts the run before printing.
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
    # median of >= 50 steps after 10 warm-up steps
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--chars", type=int, default=200)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the C4 (VCTK training) and C5 (free-running inference) lines")
    ap.add_argument("--extra-steps", type=int, default=10)
    ap.add_argument("--no-roofline", action="store_true",
                    help="skip the attention-kernel probe (profiling runs of the step alone)")
    ap.add_argument("--cpu-baseline-batch", type=int, default=2)
    ap.add_argument("--cpu-baseline-steps", type=int, default=4)
    ap.add_argument("--cpu-baseline-c2-steps", type=int, default=1,
                    help="steps of the C2-shape (B=32) CPU oracle leg, 0 = skip")
    ap.add_argument("--attn-tile", type=int, default=32)
    ap.add_argument("--pipeline-chunk", type=int, default=40,
                    help="decoder steps per chunk of the multi-stream recurrence pipeline (0 = off)")
    ap.add_argument("--plumbing", action="store_true",
                    help="CPU-only launcher check (gloo): each rank times the per-step exchange "
                         "of the real arena size instead of the training step (tests only)")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """``bench.py --gpus N`` run without an outer launcher: start N rank processes through
    torch.distributed.run (127.0.0.1 rendezvous) as a CHILD process -- this process has not
    touched the GPU and never execs -- and return its exit code.  Rank 0 prints the one JSON
    line (max-over-ranks timing); its stdout is this process's stdout."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "16")
    return subprocess.run(cmd, env=env).returncode


def plumbing(args, world: int, rank: int) -> None:
    """--plumbing: the launcher / rendezvous / max-over-ranks / JSON-line path on CPU (gloo).
    Each rank runs the per-step exchange (dp.exchange) over an arena of the LJSpeech model's
    exchange size; the line is labelled as such and is not a throughput of the training step."""
    from sat_amd import dp, hparams, params
    from sat_amd.model import BNState
    hp = hparams.ljspeech_hparams()
    n_p, n_bn = params.Layout(params.param_specs(hp)).num_params, BNState.numel(hp)
    arena = torch.zeros(n_p + n_bn + 16)
    health = torch.zeros(16, dtype=torch.int32)
    ex = lambda: dp.exchange(arena, health, arena[n_p:n_p + n_bn], arena[n_p + n_bn:])  # noqa
    for _ in range(args.warmup):
        ex()
    torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ex()
    torch.distributed.barrier()
    dt = dp.max_over_ranks(time.perf_counter() - t0, "cpu")
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": None, "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "plumbing: CPU gloo exchange of the model's arena only (no training step)",
            "config": {"workload": "launcher check", "global_batch": args.batch * world,
                       "per_gpu_batch": args.batch, "parallelism": f"dp{world}",
                       "exchange_floats": int(arena.numel())}}), flush=True)


class _Recorder:
    """Keeps the keyword arguments of the last sat_decoder_attention_fwd call (the graph-captured
    training step's own buffers), so the probe can re-launch that exact kernel afterwards."""

    def __init__(self):
        from sat_amd import kernels as K
        self.K, self.orig, self.kw = K, K.decoder_attention_fwd, None
        K.decoder_attention_fwd = self

    def __call__(self, **kw):
        self.kw = dict(kw)
        self.orig(**kw)


def attention_probe(rec, B, N, reps=6):
    """Average duration of the persistent decoder attention kernel (dec_attn_fwd_kernel: all T'
    steps of attention RNN + query + dual-source attention in one launch), timed with HIP events
    on the stream it is launched on, re-launched on the training step's own buffers after the
    timed region; and its algorithmic bytes per launch (SURVEY.md 8(d) per-step attention bytes
    times T')."""
    kw = rec.kw
    if kw is None:
        return None
    T = int(kw["T"])
    for _ in range(2):
        rec.orig(**kw)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()        # kernels.py launches on torch's current stream
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(reps):
        rec.orig(**kw)
    ev1.record(stream)
    torch.cuda.synchronize()
    avg_s = ev0.elapsed_time(ev1) / 1e3 / reps
    D1, M1, D2, M2, F, KW, U = (int(kw[k]) for k in ("D1", "M1", "D2", "M2", "F", "KW", "U"))
    f = 4  # fp32
    # per decoder step 4 (549 B N + 67,191) bytes = K1/V1/K2/V2 + the two
    # alignment states of every utterance + the attention's own weights (query, location, v)
    # (d_q = U = 256 query rows: the query layers are [U, D1] and [U, D2])
    attn_step = f * (B * N * (D1 + M1 + D2 + M2 + 5) + U * (D1 + D2)
                     + F * (KW + 1) + F * D1 + 2 * D1 + D2)
    bytes_launch = T * attn_step
    achieved = bytes_launch / avg_s / 1e9
    traffic, pmc_src = _pmc_traffic()
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": "dec_attn_fwd8_kernel (sat_decoder_attention_fwd, persistent, T' steps)",
            "bytes_per_launch": int(bytes_launch), "attn_bytes_per_step": int(attn_step),
            "steps_per_launch": T, "avg_launch_us": round(avg_s * 1e6, 1),
            "us_per_step": round(avg_s * 1e6 / T, 3), "launches_timed": reps,
            "note": "achieved = SURVEY 8(d) ALGORITHMIC attention bytes (4(549 B N + 67191) per "
                    "decoder step: K1/V1/K2/V2, alignment states, attention weights) x T' / "
                    "HIP-event launch time on the launching stream; the kernel keeps K/V slices "
                    "in LDS, so its real memory traffic (traffic = per-launch FETCH_SIZE + "
                    f"WRITE_SIZE, {pmc_src}) is lower: it is bound by its in-kernel hand-off "
                    "latency, not by HBM"}


def _pmc_traffic():
    """Per-launch memory-side bytes of the persistent attention kernel from the newest committed
    PMC summary (profiles/rNN_dec_attn_fwd_pmc.json, made by tools/pmc_persistent.py +
    tools/pmc_summary.py)."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                          "r*_dec_attn_fwd_pmc.json")))
    if not files:
        return None, "no PMC summary"
    try:
        d = json.load(open(files[-1]))
        return int(d["hbm_bytes_per_launch"]), os.path.basename(files[-1])
    except (OSError, ValueError, KeyError):
        return None, "unreadable PMC summary"


def cpu_baseline(hp, args, B=None, steps=None):
    """The CPU oracle (float32 PyTorch-CPU restatement, test infrastructure) timed on this box's
    host cores on a bounded sample of the same workload: by default C1 = LJSpeech B=2 x
    (200 chars, 1000 frames) full training steps (forward + autograd BPTT + Adam); with
    B = 32, one step of the C2 shape itself."""
    from oracle import sat_oracle as O
    from sat_amd import data, params
    B = args.cpu_baseline_batch if B is None else B
    nsteps = args.cpu_baseline_steps if steps is None else steps
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
    for s in range(nsteps):
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
    dt = (time.perf_counter() - t0) / nsteps
    return {"value": round(B * args.frames / dt, 2), "unit": "frames/s",
            "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"CPU oracle (float32 PyTorch-CPU restatement, not TF1.x), LJSpeech B={B} x "
                      f"{args.chars} chars x {args.frames} frames, {nsteps} "
                      f"full training step(s) (fwd + BPTT + Adam), {dt:.2f} s/step"}


def c4_vctk_training(args):
    """C4 (BASELINE configs[3]): VCTK multi-speaker self-attention-tacotron.json (speaker
    embedding 152 x 16 + MultiSpeakerPreNet), batch 32, teacher-forced training step, graphed."""
    from sat_amd import data, engine, hparams, train
    hp = hparams.vctk_hparams()
    B, N, T = args.batch, args.chars, args.frames
    m = engine.Tacotron(hp, "cuda", seed=4321)
    b = data.synthetic_batch(hp, B, N=N, T=T, shape="max", seed=77)
    batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
    tr = train.Trainer(m, B, N, T // hp.outputs_per_step, seed=99)
    g = train.GraphedStep(tr, batch, warmup=1)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.extra_steps):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.extra_steps
    tr.check_health(wait=True)
    out = {"metric": "teacher-forced mel frames/sec, VCTK multi-speaker batch=32, 1 MI355X",
           "value": round(B * T / dt, 1), "unit": "frames/s", "ms_per_step": round(1e3 * dt, 3),
           "steps": args.extra_steps, "config": {"workload": "VCTK self-attention-tacotron.json "
                                                 "teacher-forced training step, configs[3]",
                                                 "batch": B, "chars": N, "mel_frames": T}}
    del g, tr, m
    torch.cuda.empty_cache()
    return out


def c5_free_running(args, B=8, steps=500):
    """C5 (BASELINE configs[4]): LJSpeech free-running inference, batch 8, 500 decoder steps
    (no early stop: min_iters = max_iters), the step loop captured as hipGraphs of 25 steps."""
    from sat_amd import data, engine, hparams
    from sat_amd.inference import FreeRunningDecoder
    hp = hparams.ljspeech_hparams()
    m = engine.Tacotron(hp, "cuda", seed=1234)
    b = data.synthetic_batch(hp, B, N=args.chars, T=args.frames, shape="max", seed=55)
    batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
    dec = FreeRunningDecoder(m, max_iters=steps, min_iters=steps, check_every=25, graphs=True)
    out = dec.run(batch)                           # builds the plan and captures the graphs
    assert out["steps"] == steps
    torch.cuda.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        dec.run(batch)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    r = hp.outputs_per_step
    res = {"metric": "free-running mel frames/sec, LJSpeech batch=8, 500 decoder steps, 1 MI355X",
           "value": round(B * steps * r / dt, 1), "unit": "frames/s",
           "ms_per_decode": round(1e3 * dt, 2), "us_per_decoder_step": round(1e6 * dt / steps, 1),
           "config": {"workload": "predict_mel.py path (encoder + stop-token decoder, KV-cached "
                                  "decoder self-attention), configs[4]", "batch": B,
                      "chars": args.chars, "decoder_steps": steps, "hip_graph": True}}
    del dec, m
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.plumbing:
        torch.distributed.init_process_group("gloo")
        plumbing(args, world, rank)
        torch.distributed.destroy_process_group()
        return
    torch.cuda.set_device(local)
    dist = world > 1
    if dist:
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    from sat_amd import data, dp, engine, hparams, train
    hp = hparams.ljspeech_hparams()
    B, N, T = args.batch, args.chars, args.frames
    rec = _Recorder()
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
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(args.steps):
        run()
        evs[i + 1].record()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    dt = dp.max_over_ranks(dt, "cuda")
    step_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
    # a step the health guard skipped (hand-off timeout, id out of range) voids the number
    trainer.check_health(wait=True)
    loss1 = float(trainer.last_loss.item())
    frames = world * B * T * args.steps
    value = frames / dt
    roof = None if args.no_roofline else attention_probe(rec, B, N)
    extra = {}
    if rank == 0 and world == 1 and not args.no_extra:
        extra["c4_vctk_training"] = c4_vctk_training(args)
        extra["c5_free_running"] = c5_free_running(args)
    if rank == 0:
        cpu = None if args.no_cpu_baseline else cpu_baseline(hp, args)
        cpu_c2 = (None if args.no_cpu_baseline or args.cpu_baseline_c2_steps <= 0
                  else cpu_baseline(hp, args, B=B, steps=args.cpu_baseline_c2_steps))
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
            "median_ms_per_step": round(float(np.median(step_ms)), 3),
            "roofline": roof, "cpu_baseline": cpu, "cpu_baseline_c2": cpu_c2, **extra,
            "loss_first_timed": round(loss0, 5), "loss_last": round(loss1, 5),
        }
        print(json.dumps(line), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
