"""Throughput benchmark of the MI355X Whisper hot path (BASELINE.json metric: real-time factor,
audio-seconds / wall-second, Whisper-large-v3-turbo, 30-s chunks, 1/2/4/8 GPUs).

One step = one batch of B 30-s windows already resident in HBM (default B=24, BASELINE configs[1]):
log-mel -> encoder (32 layers) -> cross-K/V projection -> language detection (from the SOT step) ->
greedy decode of 128 new tokens per window (EOS suppressed) with the Whisper logits
processors -> segment extraction on the host -> RCCL all-gather of the per-window token arrays (N>1).
Weights are large-v3-turbo-shaped, seeded synthetic (no checkpoints offline). Each rank processes its own
B windows (chunk data parallelism, weak scaling); value = total audio seconds of all ranks / step time.

    python bench.py [--gpus N --steps K --warmup W --batch B --decode-tokens T --no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "turbo-whisper-workspace_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BF16_DENSE_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: ~2.5 PF dense bf16
FP8_DENSE_PEAK_TFLOPS = 5000.0    # MI355X_MICROARCH.md: ~5 PF dense fp8 (MX-scaled e4m3)
HBM_PEAK_GBS = 8000.0
HBM_COPY_GBS = 6290.0  # measured float4-copy rate on MI355X (MI355X_MICROARCH.md), for context beside the spec peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=("c2", "c3", "c5"), default="c2",
                    help="c2: bf16, 24 windows/GPU (BASELINE configs[1], weak scaling); c3: one full "
                         "TurboTranscriber call on 1 h of audio (120 x 30 s windows) sharded over the ranks "
                         "(configs[2], strong scaling); c5: MX fp8 encoder + bf16 decoder, 64 windows/GPU "
                         "(configs[4], weak scaling)")
    ap.add_argument("--c3-share", type=int, default=1,
                    help="c3 at one GPU: transcribe 1/R of the hour (the share one rank of R gets) instead of all "
                         "of it (a per-rank measurement; value is then that share's audio seconds / time)")
    ap.add_argument("--sub-batch-min", type=int, default=0,
                    help="c3: TurboTranscriber.sub_batch_min (split a one-batch share into two; 0 = the default)")
    ap.add_argument("--batch", type=int, default=0, help="windows per GPU (default 24 for c2, 64 for c5)")
    ap.add_argument("--decode-tokens", type=int, default=128)
    ap.add_argument("--model", default="large-v3-turbo")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--force-collective", action="store_true",
                    help="N = 1: run the RCCL path anyway (an nccl group of one; the per-batch token all-gather, c3's "
                         "waveform broadcast and sharded call)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--profile-only", action="store_true", help="warmup + steps only (for rocprofv3)")
    ap.add_argument("--eos", action="store_true",
                    help="free-running decode (SURVEY §8d, reported separately): EOS not suppressed, each window stops "
                         "at its EOS or after --decode-tokens; the roofline accounting's fixed length is the default")
    return ap.parse_args()


def launch_plan(gpus: int, env) -> str:
    """How this process runs `--gpus gpus`: "run" (it is one of the ranks, or the only one), "spawn" (no launcher
    started it and gpus > 1: start one worker per GPU through torch.distributed.run before anything touches the GPU,
    then exit with their code), or "mismatch" (a launcher started WORLD_SIZE ranks that differ from --gpus)."""
    if gpus < 1:
        return "mismatch"
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "spawn" if gpus > 1 else "run"
    return "run" if int(ws) == gpus else "mismatch"


def spawn_workers(gpus: int, argv) -> int:
    """One worker process per GPU (torchrun, rendezvous on 127.0.0.1); returns their exit code. The parent never
    initialises the GPU (no HIP call happens before this), and it starts the launcher as a child, never exec()s."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    return subprocess.run(cmd).returncode


def main():
    a = parse()
    plan = launch_plan(a.gpus, os.environ)
    if plan == "mismatch":
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE')}", file=sys.stderr)
        sys.exit(2)
    if plan == "spawn":
        sys.exit(spawn_workers(a.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU over RCCL; TW_DIST_BACKEND=gloo is a rehearsal of the multi-rank control path on fewer GPUs
    # than ranks (ranks share the cards round-robin; the numbers are then not a scaling measurement)
    backend = os.environ.get("TW_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    forced = world == 1 and a.force_collective
    if forced:  # an RCCL group of one: the per-batch all-gather runs on device tensors exactly as at N > 1
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", local))

    from twamd.config import PRESETS, GenerationSettings
    from twamd.engine import WhisperEngine
    from twamd.synth_audio import workload
    from twamd.weights import build_weights

    dims = PRESETS[a.model]
    gen = GenerationSettings.default(dims)
    fp8 = a.config == "c5"
    strong = a.config == "c3"
    if strong:  # engine batches of <= 24 windows; a rank's share of the 120 windows is cut by pipeline.batch_sizes
        B = a.batch or 24
    else:
        B = a.batch or (64 if fp8 else 24)
    T = a.decode_tokens
    if strong:  # the product call path: TurboTranscriber (ASR-pipeline signature) over the engine
        from twamd.pipeline import TurboTranscriber
        tr = TurboTranscriber.from_pretrained(a.model, seed=1234, max_batch=B, device=f"cuda:{local}", max_beams=1)
        if a.sub_batch_min:
            tr.sub_batch_min = a.sub_batch_min
        eng = tr.engine
    else:
        w = build_weights(dims, seed=1234)
        eng = WhisperEngine(w, gen, max_batch=B, device=f"cuda:{local}", enc_fp8=fp8)
    dom = "gemm_mx" if fp8 else "gemm_big"
    peak = FP8_DENSE_PEAK_TFLOPS if fp8 else BF16_DENSE_PEAK_TFLOPS
    if not a.eos:
        eng.set_suppress_tokens(list(gen.suppress_tokens) + [gen.special.eot])  # fixed decode length
    from twamd import dist as twd
    if forced:
        twd.FORCE_COLLECTIVE = True
    if strong:
        # 1 h of synthetic speech-like audio (120 seeded 30-s windows back to back), on the host as a caller's array
        hour = workload(120 // max(1, a.c3_share), 30.0, seed=1234).reshape(-1)
        call_kw = dict(chunk_length_s=30, stride_length_s=0, batch_size=B, return_timestamps=True,
                       generate_kwargs={"task": "transcribe", "num_beams": 1, "max_new_tokens": T, "max_passes": 1})
    else:
        audio = workload(B, 30.0, seed=1234 + 1000 * rank)
        eng.wave[:B].copy_(torch.from_numpy(audio))

    def run(n_steps):
        if strong:  # one step = one full call: host waveform -> broadcast -> shard -> batches -> gather -> text
            out = None
            for _ in range(n_steps):
                out = tr(hour, **call_kw)
            return [p for w in tr.last_window_passes for p in w[:1]] if out is not None else []
        """n_steps batches of B windows through the engine's two-slot pipeline (the encoder of batch k+1 runs on
        a second HIP stream beside the decode of batch k); every rank then all-gathers each batch's tokens."""
        res = eng.run_batches([B] * n_steps, task="transcribe", max_new_tokens=T, max_passes=1)
        if world > 1 or forced:  # rank r holds windows [rB, (r+1)B) of each batch: one RCCL all-gather per batch
            res = [twd.gather_tokens(seqs, lg, world * B)[0] for seqs, lg in zip(res, eng.batch_langs)]
        return res[-1] if res else []

    run(a.warmup)
    extra_warm = 0
    if not strong and a.warmup > 0:
        # captured decode graphs are keyed by pipeline slot (the cross-K/V pointer they bake) and by whether an encoder
        # chunk runs beside the pass (its own kernel choices, engine._dec_context): batch k of a run decodes beside the
        # next batch's encoder in slot k % 2, the last one alone in slot (n - 1) % 2. A warmup that did not meet every
        # (beside/alone, slot) the timed run meets leaves graph captures inside the timed region (~3.7 ms per step at
        # K = 20, W = 5; ~15 ms at the defaults: profiles/r05ai_bench_bisect.txt): up to 4 more untimed batches then.
        extra_warm = warmup_completion(a.steps, a.warmup)
        if extra_warm:
            run(extra_warm)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # HIP events around every launch of the dominant kernel (k_gemm_big) on the engine stream, inside the
    # timed region (the encoder is not graph-captured; ~0.3 us per event against 0.2-1 ms per launch)
    # (TW_BENCH_EXTRA_FAMILIES="attn_encoder,...": further families timed the same way and listed in kernel_families)
    extra = {f for f in os.environ.get("TW_BENCH_EXTRA_FAMILIES", "").split(",") if f}
    eng.timers, eng.timer_families = ({}, {dom} | extra) if os.environ.get("TW_BENCH_TIMERS", "1") != "0" else (None, None)
    t0 = time.perf_counter()
    seqs = run(a.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    fam = eng.timer_summary()
    eng.timers, eng.timer_families = None, None
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=eng.device if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if a.profile_only:
        if rank == 0:
            print(json.dumps({"profile_only": True, "ms_per_step": 1000 * dt / a.steps}))
        return
    ms = 1000.0 * dt / a.steps
    audio_s = (120 // max(1, a.c3_share)) * 30.0 if strong else world * B * 30.0
    rtf = audio_s / (dt / a.steps)
    n_tok = [len(s) for s in seqs]

    # dominant kernel: all k_gemm_big launches of the timed steps (every epilogue variant)
    dfam = [v for k, v in fam.items() if k[0] == dom]
    n_l = max(1, sum(v[0] for v in dfam))  # (0 with TW_BENCH_TIMERS=0: A/B runs without events)
    work = sum(v[1] for v in dfam)
    tot_ms = sum(v[2] for v in dfam)
    avg_ms = max(tot_ms / n_l, 1e-9)
    achieved = (work / n_l) / (avg_ms * 1e-3) / 1e12
    families = {f"{k[0]}<{k[1]}>": {"launches": v[0], "tflop": round(v[1] / 1e12, 3), "ms": round(v[2], 3),
                                    "tflops": round(v[1] / (v[2] * 1e-3) / 1e12, 1) if v[2] > 0 else None}
                for k, v in fam.items()}
    # the bf16 family runs as k_gemm_big beside a decode and as k_gemm_8p alone (engine._set_gemm_context)
    # (the MX family: k_gemm_8p_mx on every encoder shape since round 5, k_gemm_mx before and on request)
    fam_k = ("k_gemm_mx", "k_gemm_8p_mx") if fp8 else ("k_gemm_big", "k_gemm_8p", "k_gemm_8pp")
    traffic, traffic_src = measured_traffic(fam_k, fp8)
    mfma_busy, mfma_src = measured_mfma(fam_k, fp8)

    # secondary (HBM-bound) kernel: decoder cross-attention, timed on one eager decode pass outside the timed
    # region (the timed decode steps replay a hipGraph, which has no room for events)
    dec = decode_cross_roofline(eng, B, traffic_lookup=measured_traffic(("k_attn_decode_cross",), fp8))

    out = {
        "metric": "real-time factor (audio-sec/wall-sec) Whisper-v3-turbo, 30s chunks, 1/2/4/8 GPU",
        "value": round(rtf, 1),
        "unit": "audio-s/wall-s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "warmup_extra_batches": extra_warm,  # (untimed: completes the decode-graph captures, see above)
        "ms_per_step": round(ms, 2),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "fp8-e4m3 (MX) encoder projections + bf16" if fp8 else "bf16",
        "data": "synthetic (seeded speech-like 16 kHz audio, 10% silent windows; seeded synthetic weights)",
        "config": {"workload": f"whisper-{a.model} {'MX-fp8 encoder + bf16 decoder' if fp8 else 'bf16'}, "
                               + (f"one TurboTranscriber call on {audio_s / 3600:g} h of host audio "
                                  f"({int(audio_s // 30)} x 30s windows, chunk_length_s=30, stride 0) sharded over "
                                  f"the GPUs, engine batches of <= {B} (sub-batches: "
                                  f"{tr.sub_batch_min or 'off'}), " if strong else
                                  f"batch={B} x 30s windows per GPU, ")
                               + (f"greedy, free-running (EOS allowed, at most {T} new tokens/window), one seek "
                                  "pass, timestamps on, language detected" if a.eos else
                                  f"greedy, {T} new tokens/window (EOS suppressed, one seek pass), timestamps on, "
                                  "language detected"),
                   "c3_share": a.c3_share if strong else None,
                   "collectives": ("rccl" if backend == "nccl" else backend) if world > 1 else
                                  ("rccl (group of one, forced)" if forced else "none"),
                   "global_batch": int(audio_s // 30), "seq_len": 3000, "parallelism": f"chunk-dp{world}",
                   "decode_tokens_per_window": T, "mean_tokens_out": float(np.mean(n_tok))},
        "roofline": {"bound": "mfma",
                     "kernel": ("k_gemm_8p_mx / k_gemm_mx (encoder q/k/v/o + fc1/fc2, MX fp8 MFMA)" if fp8 else
                                "k_gemm_big / k_gemm_8p / k_gemm_8pp (all encoder/conv/cross-KV projections, bf16 MFMA)"),
                     "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": traffic,
                     "traffic_source": traffic_src, "mfma_busy_pct": mfma_busy, "mfma_source": mfma_src,
                     "launches_per_step": n_l // a.steps,
                     "avg_launch_ms": round(avg_ms, 4), "flop_per_launch": work / n_l},
        "roofline_decode": dec,
        "parity": None,
        "kernel_families": families,
        "cpu_baseline": None,
    }
    if rank == 0:
        out["parity"], out["parity_detail"] = (parity_vs_golden(eng, B, T, a.model, fp8) if not strong and not a.eos else
                                               (None, {"skipped": "free-running decode: the golden is the EOS-suppressed "
                                                                  "decode"}) if a.eos else
                                               (None, {"skipped": "c3 windows differ from the golden's; the same "
                                                                  "engine's parity is the c2 line's"}))
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(dims, gen, T, a.cpu_threads)
    if rank == 0:
        print(json.dumps(out))
    if world > 1 or forced:
        dist.destroy_process_group()


def parity_vs_golden(eng, B, T, model, fp8):
    """Rank 0's last timed batch against transformers' fp32 decode of the same seeded weights and audio:
    free_decode — windows 0 (speech) and 23 (silent) as decoded in the timed region (tests/golden/turbo.npz): tokens
    equal, or diverging first at a near-tie within TAU = 0.15 logits; language ids equal. teacher_forced — 6 windows
    (turbo_bench.npz) at all 128 positions: each fp32 sequence fed through the same captured B = 24 decode after the
    timed region, top-16 logits within LOGIT_ABS, argmax and timestamp-rule margin within TAU at every position
    (turbo_parity.forced_decode). Only the bf16 config-2 workload (24 windows, 128 tokens) has a golden; anything
    else reports None."""
    if T != 128 or model != "large-v3-turbo" or B != (64 if fp8 else 24):
        return None, {"skipped": "no fp32 golden for this workload"}
    if fp8:  # config 5: windows 0, 5, 11, 17 of its 64 hold the same seeded clips as config 2's (turbo_bench.npz)
        try:
            sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
            import turbo_parity as tp

            forced = tp.forced_decode(eng, tp.load_bench(), B, T, windows=(0, 5, 11, 17), fp8=True)
        except Exception as e:  # reported, never allowed to sink the GPU number
            return False, {"error": repr(e)[:200]}
        return forced["ok"], {"reference": "transformers fp32 CPU, tests/golden/turbo_bench.npz (the same seeded "
                                           "clips as windows 0, 5, 11, 17 of this batch)",
                              "bounds": "MX-fp8 encoder: turbo_parity.FP8_* (stated, fixed)", "teacher_forced": forced,
                              "positions_checked": forced["positions_checked"],
                              "worst_d_logit": forced["worst_d_logit"]}
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        import turbo_parity as tp

        z = tp.load()
        passes, langs = eng.batch_passes[-1], eng.batch_langs[-1]
        det = {f"window{w}": tp.check_bench_window(z, w, passes[w][0], langs[w]) for w in tp.BENCH_WINDOWS}
        # every position: the fp32 sequences of 6 windows teacher-forced through the same captured B = 24 decode
        # (after the timed region, on the same engine and resident waveforms)
        forced = tp.forced_decode(eng, tp.load_bench(), B, T)
    except Exception as e:  # reported, never allowed to sink the GPU number
        return False, {"error": repr(e)[:200]}
    ok = all(r["lang_ok"] and r["status"] in ("exact", "within_tau") for r in det.values()) and forced["ok"]
    return ok, {"tau": tp.TAU, "reference": "transformers fp32 CPU, tests/golden/turbo.npz + turbo_bench.npz",
                "free_decode": det, "teacher_forced": forced, "positions_checked": forced["positions_checked"],
                "worst_d_logit": forced["worst_d_logit"]}


def decode_graph_keys(n: int) -> set:
    """The captured decode graphs a run_batches call of n batches meets: batch k decodes beside the next batch's
    encoder in pipeline slot k % 2, the last batch alone in slot (n - 1) % 2 (engine graph keys carry the slot and the
    pass context)."""
    return {("beside", k % 2) for k in range(n - 1)} | ({("alone", (n - 1) % 2)} if n else set())


def warmup_completion(steps: int, warmup: int) -> int:
    """Untimed batches to run after the warmup so that every decode graph the timed run of `steps` batches meets has
    been captured (0 if the warmup already met them all, or when there is no warmup)."""
    if warmup <= 0:
        return 0
    need, have = decode_graph_keys(steps), decode_graph_keys(warmup)
    if need <= have:
        return 0
    return next(n for n in range(1, 5) if need <= have | decode_graph_keys(n))


def profile_order(path: str):
    """Sort key of a profiles/ file by its round tag: (round, tag length, tag) — r05b < r05z < r05ab < r06a. A plain
    basename sort put r04t after r04ae (and would put r05b after r05ab)."""
    import re

    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    if not m:
        return (-1, 0, os.path.basename(path))
    return (int(m.group(1)), len(m.group(2)), m.group(2))


def measured_traffic(kernels, c5: bool = False):
    """HBM bytes per launch of the `kernels` (names of one family, launch-weighted together) from the newest
    rocprofv3 PMC summary under profiles/ that has any of them (scripts/summarize_prof.py: 2*FETCH_SIZE + WRITE_SIZE
    per launch), or (None, None). Config-5 runs (--config c5) write *_c5_traffic.json; each config reads only its
    own."""
    import glob

    # newest = the latest round tag (profile_order); file mtimes do not survive the copy to the GPU box reliably
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic.json")), key=profile_order)
    files = [f for f in files if ("_c5_" in os.path.basename(f)) == c5]
    for f in reversed(files):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        hit = [d[k] for k in kernels if k in d and d[k].get("hbm_bytes") and d[k].get("launches")]
        if hit:
            n = sum(h["launches"] for h in hit)
            return sum(h["hbm_bytes"] * h["launches"] for h in hit) / n, os.path.relpath(f, ROOT)
    return None, None


def measured_mfma(kernels, c5: bool = False):
    """MFMA busy % of the dominant family's launches from the newest profiles/*mfma.json (scripts/summarize_prof.py:
    rocprofv3 PMC pass, SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE per XCD x 1024 SIMDs; dispatches serialised by
    the profiler, so this is the kernel's own utilisation, not the in-situ one), launch-weighted, or (None, None)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*mfma.json")), key=profile_order)
    files = [f for f in files if ("_c5_" in os.path.basename(f)) == c5]
    for f in reversed(files):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        hit = [d[k] for k in kernels if k in d and d[k].get("launches")]
        if hit:
            n = sum(h["launches"] for h in hit)
            return round(sum(h["mfma_util_pct"] * h["launches"] for h in hit) / n, 1), os.path.relpath(f, ROOT)
    return None, None


def decode_cross_roofline(eng, B, traffic_lookup):
    """k_attn_decode_cross achieved HBM GB/s on one eager decoder step (4 launches)."""
    saved = eng.use_graphs
    try:
        eng.timers, eng.timer_families = {}, {"attn_decode_cross"}
        eng.decoder_step(B)
        fam = eng.timer_summary()
    finally:
        eng.timers, eng.timer_families, eng.use_graphs = None, None, saved
    (n_l, work, tot_ms), = fam.values()
    gbs = (work / n_l) / (tot_ms / n_l * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": "k_attn_decode_cross", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic_lookup[0],
            "bytes_per_launch": work / n_l, "avg_launch_ms": round(tot_ms / n_l, 4),
            # the chip's measured streaming ceiling (MI355X_MICROARCH.md: a float4 copy reaches 6.29 TB/s)
            "copy_peak": HBM_COPY_GBS, "frac_of_copy": round(gbs / HBM_COPY_GBS, 4)}


def _cgroup_cpus():
    """The CPU quota of this process's cgroup (cgroup v2 cpu.max: quota / period), or None without one."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        return None


def host_threads() -> int:
    """Threads for the CPU baseline: every CPU this process may run on (its affinity mask), bounded by the cgroup's
    CPU quota and by OMP_NUM_THREADS when the box sets it (the GPU box's share is 16 of a larger machine: more
    threads than the quota only time-slice)."""
    n = len(os.sched_getaffinity(0))
    for lim in (_cgroup_cpus(), os.environ.get("OMP_NUM_THREADS")):
        if lim:
            n = min(n, int(lim))
    return max(1, n)


def host_cpu_report() -> dict:
    return {"affinity": len(os.sched_getaffinity(0)), "cgroup_quota": _cgroup_cpus(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "os_cpu_count": os.cpu_count()}


def cpu_baseline(dims, gen, T, threads):
    """The reference's executed transcription path (transformers ASR pipeline, what
    vocalis/core/audio_pipeline.py:351-358 calls) on the host CPU, fp32, same seeded weights, with the reference's
    kwargs (chunk_length_s=60, stride_length_s=5, batch_size=32, task=transcribe, return_timestamps=True) on a
    bounded sample: 210 s of speech-like audio = 4 windows of the 60/5 windowing, T new tokens per window (EOS
    suppressed, as on the GPU), one seek pass per window. Timed twice on one pipeline object: num_beams=1 (the
    parity decode; `value`) and the pipeline's as-shipped default num_beams=5."""
    import copy
    import platform

    from oracle import hf_baseline
    from twamd.synth_audio import speech_like

    threads = threads or host_threads()
    g = copy.deepcopy(gen)
    g.suppress_tokens = list(gen.suppress_tokens) + [gen.special.eot]
    audio = speech_like(210.0, 1234)
    runs = {}
    try:
        t0 = time.perf_counter()
        pipe = hf_baseline.build_pipeline(dims, g, 1234, threads)
        build_s = time.perf_counter() - t0
        for nb in (1, 5):
            runs[nb] = hf_baseline.time_reference(dims, g, audio, max_new_tokens=T, threads=threads, num_beams=nb,
                                                  one_pass=True, pipe=pipe)
    except Exception as e:  # the baseline is reported, never allowed to sink the GPU number
        return {"value": None, "error": repr(e)[:200], **({"greedy_wall_s": runs[1]["wall_s"]} if 1 in runs else {})}
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), cpu)
    except OSError:
        pass
    r1, r5 = runs[1], runs[5]
    return {"value": round(r1["audio_s"] / r1["wall_s"], 3), "unit": "audio-s/wall-s", "cores": threads,
            "kind": "reference", "cpu": cpu, "host_cpus": host_cpu_report(),
            "as_shipped_beam5": {"value": round(r5["audio_s"] / r5["wall_s"], 3), "wall_s": round(r5["wall_s"], 2)},
            "sample": f"transformers {__import__('transformers').__version__} ASR pipeline fp32 on CPU (the path the "
                      f"reference executes) with the reference kwargs (chunk_length_s=60, stride_length_s=5, "
                      f"batch_size=32, task=transcribe, return_timestamps=True) on 210 s of audio = 4 windows (the 60/5 "
                      f"windowing feeds each window's first 30 s to the model, SURVEY §0.3, so per window of model work "
                      f"this rate is 210/120 of a 30-s-mode rate); {T} new "
                      f"tokens per window (EOS suppressed), one seek pass; value = num_beams=1 (wall "
                      f"{r1['wall_s']:.1f}s), as_shipped_beam5 = the pipeline default num_beams=5; weights built in "
                      f"{build_s:.0f}s (untimed)"}


if __name__ == "__main__":
    main()
