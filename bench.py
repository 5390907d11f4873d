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
    ap.add_argument("--no-ragged", action="store_true",
                    help="skip the drop-in model_fn path over ragged TFRecord batches")
    ap.add_argument("--no-fallback", action="store_true",
                    help="skip the B=64 per-step-path (persistent-ineligible) extra line")
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
    """Keeps the keyword arguments of the last call of one persistent-kernel entry
    (``kernels.decoder_attention_fwd`` / ``_bwd``: the graph-captured training step's own
    buffers), so the probe can re-launch that exact kernel afterwards."""

    def __init__(self, name):
        from sat_amd import kernels as K
        self.K, self.name, self.orig, self.kw = K, name, getattr(K, name), None
        setattr(K, name, self)

    def __call__(self, **kw):
        self.kw = dict(kw)
        self.orig(**kw)


def _attn_fwd_step_bytes(kw, B, N):
    """per decoder step 4 (549 B N + 67,191) bytes = K1/V1/K2/V2 + the two
    alignment states of every utterance + the attention's own weights (query, location, v)
    (d_q = U = 256 query rows: the query layers are [U, D1] and [U, D2])."""
    D1, M1, D2, M2, F, KW, U = (int(kw[k]) for k in ("D1", "M1", "D2", "M2", "F", "KW", "U"))
    return 4 * (B * N * (D1 + M1 + D2 + M2 + 5) + U * (D1 + D2)
                + F * (KW + 1) + F * D1 + 2 * D1 + D2)


def _attn_bwd_step_bytes(kw, B, N):
    """The BPTT's per-step algorithmic bytes: the forward's 8(d) set
    (memories, alignment states, attention weights) + the energy-tanh history it re-reads
    (ZH, B N (D1 + D2)) + the energy / location-feature gradients it writes (DE1, DE2, DFH:
    B N (2 + F))."""
    D1, D2, F = (int(kw[k]) for k in ("D1", "D2", "F"))
    return _attn_fwd_step_bytes(kw, B, N) + 4 * B * N * ((D1 + D2) + 2 + F)


def _roof(bytes_launch, avg_s, T, reps, kernel, note, traffic=None, pmc_src=None):
    achieved = bytes_launch / avg_s / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": pmc_src, "kernel": kernel, "bytes_per_launch": int(bytes_launch),
            "attn_bytes_per_step": int(bytes_launch // T), "steps_per_launch": T,
            "avg_launch_us": round(avg_s * 1e6, 1), "us_per_step": round(avg_s * 1e6 / T, 3),
            "launches_timed": reps, "note": note}


def attention_probe(rec, B, N, reps=6):
    """Average duration of the persistent decoder attention kernel (dec_attn_fwd8_kernel: all T'
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
    traffic, pmc_src = _pmc_traffic("dec_attn_fwd", "decoder_persistent8.hip")
    return _roof(T * _attn_fwd_step_bytes(kw, B, N), avg_s, T, reps,
                 "dec_attn_fwd8_kernel (sat_decoder_attention_fwd, persistent, T' steps)",
                 "achieved = SURVEY 8(d) ALGORITHMIC attention bytes (4(549 B N + 67191) per "
                 "decoder step: K1/V1/K2/V2, alignment states, attention weights) x T' / "
                 "HIP-event launch time on the launching stream; the kernel keeps K/V slices "
                 "in LDS, so its real memory traffic (traffic = per-launch FETCH_SIZE + "
                 "WRITE_SIZE of the PMC summary named in traffic_source) is lower: it is bound "
                 "by its in-kernel hand-off latency, not by HBM", traffic, pmc_src)


def attention_bwd_probe(rec, B, N, reps=4):
    """The same for the attention chain's BPTT (dec_attn_bwd8_kernel), re-launched on the
    step's own buffers.  It accumulates into RD in place, so RD is restored between launches
    and every launch is bracketed by its own HIP events (the restore is outside them)."""
    kw = rec.kw
    if kw is None:
        return None
    T = int(kw["T"])
    rd = kw["RD"]
    rd0 = rd.clone()
    stream = torch.cuda.current_stream()
    times = []
    for i in range(reps + 1):
        rd.copy_(rd0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        rec.orig(**kw)
        e1.record(stream)
        torch.cuda.synchronize()
        if i:                                   # the first launch is a warm-up
            times.append(e0.elapsed_time(e1) / 1e3)
    rd.copy_(rd0)
    avg_s = float(np.mean(times))
    traffic, pmc_src = _pmc_traffic("dec_attn_bwd", "decoder_persistent8_bwd.hip")
    return _roof(T * _attn_bwd_step_bytes(kw, B, N), avg_s, T, reps,
                 "dec_attn_bwd8_kernel (sat_decoder_attention_bwd, persistent, T' reverse steps)",
                 "achieved = the forward's 8(d) bytes + the ZH energy-tanh history re-read "
                 "(B N (D1+D2) floats) + the DE1/DE2/DFH gradients written (B N (2+F)) per "
                 "step, x T' / HIP-event time of one launch", traffic, pmc_src)


def _pmc_traffic(kernel_tag: str, source: str):
    """Per-launch memory-side bytes of a persistent attention kernel from the newest committed
    PMC summary ``profiles/rNN_<kernel_tag>_pmc.json`` (tools/pmc_persistent.py +
    tools/pmc_summary.py), with the summary's provenance: its file, the sha256 of the kernel
    source it was measured on, and whether that equals the source of THIS tree (a stale summary
    is reported as such, not as this build's traffic)."""
    import glob
    import hashlib
    here = os.path.dirname(os.path.abspath(__file__))
    import re
    files = glob.glob(os.path.join(here, "profiles", f"r*_{kernel_tag}_pmc.json"))
    if not files:
        return None, {"file": None, "why": "no PMC summary committed"}

    def tag_key(path):
        # round tags are r<round><letters>: r05 < r05a < r05z < r05aa < r05ab < r06 (the
        # letters count like a spreadsheet column; a plain string sort puts r05y after r05ab)
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
        if not m:
            return (-1, -1)
        col = 0
        for ch in m.group(2):
            col = col * 26 + (ord(ch) - 96)
        return (int(m.group(1)), col)

    src = os.path.join(here, "self-attention-tacotron_amd", "csrc", source)
    try:
        now = hashlib.sha256(open(src, "rb").read()).hexdigest()[:16]
    except OSError:
        now = None
    summaries = []
    for f in files:
        try:
            d = json.load(open(f))
            summaries.append((tag_key(f), f, d, int(d["hbm_bytes_per_launch"])))
        except (OSError, ValueError, KeyError):
            continue
    if not summaries:
        return None, {"file": os.path.basename(max(files, key=tag_key)),
                      "why": "unreadable PMC summary"}
    # the newest summary measured on THIS tree's kernel source; else the newest one (stale)
    cur = [x for x in summaries if x[2].get("source_sha16") == now]
    _, f, d, nbytes = max(cur or summaries, key=lambda x: x[0])
    was = d.get("source_sha16")
    return nbytes, {"file": os.path.basename(f), "measured_on_source_sha16": was,
                    "current_source_sha16": now, "current": was == now}


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


def fallback_training(args, B=64, steps=3):
    """The persistent-eligibility cliff, measured: a per-GPU batch the
    one-launch decoder kernels cannot take (B=64 > 32: ceil(B/8) * ceil(N/32) > 32 groups)
    runs the per-step launch path with a PersistentFallbackWarning.  Same step as the headline
    (graphed, fwd + BPTT + Adam) at B=64; reported so the cost of leaving the eligible shapes
    is a number, not a surprise."""
    import warnings
    from sat_amd import data, decoder, engine, hparams, params, train
    hp = hparams.ljspeech_hparams()
    N, T = args.chars, args.frames
    why = decoder.persistent_ineligible_reason(params.resolve_dims(hp), B, N)
    try:
        m = engine.Tacotron(hp, "cuda", seed=4321)
        b = data.synthetic_batch(hp, B, N=N, T=T, shape="max", seed=78)
        batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
        tr = train.Trainer(m, B, N, T // hp.outputs_per_step, seed=98)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", decoder.PersistentFallbackWarning)
            g = train.GraphedStep(tr, batch, warmup=1)
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        tr.check_health(wait=True)
        out = {"value": round(B * T / dt, 1), "unit": "frames/s", "ms_per_step": round(1e3 * dt, 3),
               "steps": steps}
        del g, tr, m
    except Exception as e:          # reported, never fatal to the headline line
        out = {"error": f"{type(e).__name__}: {e}"[:300]}
    torch.cuda.empty_cache()
    out.update({"metric": f"teacher-forced mel frames/sec, LJSpeech batch={B} on 1 MI355X "
                          "(per-step launch path: persistent decoder not eligible)",
                "why_not_persistent": why,
                "config": {"workload": "C2 step at a per-GPU batch outside the persistent "
                                       "kernels' shapes", "batch": B, "chars": N, "mel_frames": T}})
    return out


def drop_in_ragged(args, n_batches=24, B=32, cache=32):
    """The drop-in training path measured: synthetic LJSpeech-format TFRecords
    (ljs-like: N ~ U{40..200} chars, T = min(996, 5 N + 4) frames, the reference's record
    layout preprocess/ljspeech.py:23-45) read by the dataset pipeline -- interleave, prepare
    (normalise, silence, r-rounding, done / masks), group_by_batch buckets with per-batch
    padding (datasets/ljspeech/dataset.py:126-286) -- and fed to ``model_fn`` TRAIN as a
    maintainer's loop would (host batches; the pinned upload is INSIDE the timed region).
    Three arms over the same batches: eager (graph_cache=0), the graph cache's first pass
    (every new padded shape = one eager step + a capture) and its second pass (every shape
    cached: one copy + one replay per batch).  frames = sum of B x T_pad over the batches."""
    import tempfile
    from sat_amd import datasets as D, hparams, models as MD, tfrecord as R
    hp = hparams.ljspeech_hparams()
    hp.set_hparam("average_mel_level_db", [0.0] * hp.num_mels)
    hp.set_hparam("stddev_mel_level_db", [1.0] * hp.num_mels)
    rng = np.random.default_rng(2024)
    n_utt = n_batches * B
    shards = 4
    with tempfile.TemporaryDirectory() as tmp:
        srcs, tgts = [], []
        for sh in range(shards):
            sr, tr_ = [], []
            for i in range(sh, n_utt, shards):
                n = int(rng.integers(40, 201))
                t = min(996, 5 * n + 4)
                sr.append(R.source_example(i, f"LJ{i:05d}", rng.integers(1, 71, n), "x"))
                tr_.append(R.target_example(i, f"LJ{i:05d}",
                                            rng.standard_normal((t, hp.num_mels)).astype(np.float32)))
            fs, ft = os.path.join(tmp, f"s{sh}.tfrecord"), os.path.join(tmp, f"t{sh}.tfrecord")
            R.write_tfrecords(sr, fs)
            R.write_tfrecords(tr_, ft)
            srcs.append(fs)
            tgts.append(ft)
        t0 = time.perf_counter()
        batches = list(D.DatasetSource.create_from_tfrecord_files(srcs, tgts, hp)
                       .prepare_and_zip().filter_by_max_output_length().group_by_batch(B))
        pipe_s = time.perf_counter() - t0
    batches = [x for x in batches if len(x[0].source) == B]
    frames = sum(int(l.mel.shape[0] * l.mel.shape[1]) for _, l in batches)
    shapes = {(f.source.shape[1], l.mel.shape[1]) for f, l in batches}

    def run(model):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f, l in batches:
            loss = model.model_fn(f, l, MD.ModeKeys.TRAIN, hp).loss
        torch.cuda.synchronize()
        return time.perf_counter() - t0, float(loss.item())

    out = {"metric": "teacher-forced mel frames/sec over ragged ljs-like batches through "
                     "datasets.group_by_batch -> model_fn TRAIN, batch=32, 1 MI355X",
           "unit": "frames/s", "batches": len(batches), "distinct_padded_shapes": len(shapes),
           "padded_frames": frames, "pipeline_s": round(pipe_s, 2)}
    try:
        m = MD.DualSourceSelfAttentionTacotronModel(hp, device="cuda", seed=11, graph_cache=0)
        run(m)                                          # warm-up pass (allocator, streams)
        dt, loss = run(m)
        out["eager"] = {"value": round(frames / dt, 1), "ms_per_batch": round(1e3 * dt / len(batches), 2),
                        "loss_last": loss}
        del m
        torch.cuda.empty_cache()
        m = MD.DualSourceSelfAttentionTacotronModel(hp, device="cuda", seed=11, graph_cache=cache)
        dt1, _ = run(m)
        dt2, loss = run(m)
        c = m._graphs
        out["graph_cache_first_pass"] = {"value": round(frames / dt1, 1),
                                         "ms_per_batch": round(1e3 * dt1 / len(batches), 2)}
        out["graph_cache_steady"] = {"value": round(frames / dt2, 1),
                                     "ms_per_batch": round(1e3 * dt2 / len(batches), 2),
                                     "loss_last": loss}
        out["value"] = out["graph_cache_steady"]["value"]
        out["cache"] = {"size": cache, "hits": c.hits, "misses": c.misses,
                        "evictions": c.evictions}
        del m, c
    except Exception as e:          # reported, never fatal to the headline line
        out["error"] = f"{type(e).__name__}: {e}"[:300]
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
    rec = _Recorder("decoder_attention_fwd")
    rec_bwd = _Recorder("decoder_attention_bwd")
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
    roof_bwd = None if args.no_roofline else attention_bwd_probe(rec_bwd, B, N)
    extra = {}
    if rank == 0 and world == 1 and not args.no_extra:
        extra["c4_vctk_training"] = c4_vctk_training(args)
        extra["c5_free_running"] = c5_free_running(args)
        if not args.no_ragged:
            extra["drop_in_ragged_ljs"] = drop_in_ragged(args)
        if not args.no_fallback:
            extra["fallback_b64_per_step_path"] = fallback_training(args)
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
            "roofline": roof, "roofline_bptt": roof_bwd, "cpu_baseline": cpu, "cpu_baseline_c2": cpu_c2, **extra,
            "loss_first_timed": round(loss0, 5), "loss_last": round(loss1, 5),
        }
        print(json.dumps(line), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
