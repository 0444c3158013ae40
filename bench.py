"""Benchmark: utterances/s of the full ERGM training step (forward + backward + AdamW + LR step) on
MELD-shaped synthetic batches, GPT-2-small + audio/visual fusion, batch 16 per GPU, bf16 MFMA
(BASELINE.json configs[1]; with --gpus N one process per GPU over RCCL, configs[2]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c4] [--no-cpu-baseline]

Prints ONE JSON line on rank 0.  ``value`` = all utterances processed by all ranks ÷ the max over
ranks of the wall time of exactly K steps (barrier + device sync on both sides).  ``roofline`` is the
step's dominant time class, the weight-gradient GEMMs (every Conv1D dW, the stacked caption K/V dW and
the tied LM-head dW): their algorithmic FLOPs over their in-step launch durations, from HIP event
pairs the native executor records around each launch in extra steps run right after the timed region
(``--probe 1..4`` times a single launch inside the timed steps instead); ``roofline_secondary`` is the
LM-head forward main launch; ``mfma_step`` is the whole step's algorithmic FLOPs over
the step time against the 2.5 PF/s dense bf16 peak.  ``cpu_baseline`` times the CPU oracle (fp32
PyTorch restatement of the reference step) on the host cores for a bounded sample.

Reproducible: ``torch.manual_seed(--seed)`` before the model is built fixes the dropout mask stream
(rank 0's seed is broadcast under DP), so two runs of a config print the same ``train_metrics``.
Data parallel (N > 1): the library's defaults, the reference's gradient arithmetic — an fp32 all-reduce
(one fp32 sum per element) and the replicated AdamW update.  ERGM_DP_GRAD=bf16 / ERGM_DP_ZERO=1 opt into the
bf16 exchange (narrower: every rank's gradient and the reduced sum rounded to bf16) with the sharded update;
the JSON ``config`` records both settings.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def lmhead_split_cols(T: int, Vp: int) -> int:
    """Columns of the LM head's main launch (model.cpp lmhead_split_cols): the largest multiple of 256
    whose 256x256 tiles fill whole rounds of 256 CUs; the rest runs as a small-tile tail launch."""
    rows, q = -(-T // 256), 256
    while rows % 2 == 0 and q > 1:
        rows //= 2
        q //= 2
    n0 = (Vp // 256 // q) * q * 256
    return n0 if n0 > 0 and Vp - n0 >= 256 else Vp


def pmc_traffic(key, config: str = "c2"):
    """HBM bytes per launch of the probed kernel from the newest committed PMC summary
    (profiles/r*_pmc_traffic.json, written by tools/pmc_traffic.py from separate rocprofv3
    FETCH_SIZE / WRITE_SIZE passes).  None when no summary covers the probe."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                          "r*_pmc_traffic.json")))
    if key is None or config != "c2":  # the committed PMC passes are of the C2 workload
        return None, None
    for fn in reversed(files):  # the newest summary that covers `key`
        with open(fn) as f:
            rec = json.load(f).get(key)
        if rec:
            return round(rec["hbm_bytes"]), os.path.relpath(fn, os.path.dirname(os.path.abspath(__file__)))
    return None, None
CONFIGS = {
    # name: (model, S, turns, batch per GPU, pooled feature width, fp8 forward GEMMs, description)
    "c2": ("small", 128, 5, 16, 768, False,
           "GPT-2-small + audio/visual fusion, MELD-shape (S=128, 5 turns), B=16/GPU"),
    "c4": ("small", 512, 20, 8, 768, False,
           "GPT-2-small + audio/visual fusion, IEMOCAP-shape (S=512, 20 turns), B=8/GPU, larger features: "
           "BLIP-vision [B,197,768] (row 0 injected) and wav2vec2 [B,400,768] mean-pooled on the GPU each step"),
    "c5": ("medium", 128, 5, 32, 768, True, "GPT-2-medium + 768-d audio/visual features through projection "
           "GEMMs, fp8 (e4m3) forward Conv1D GEMMs, MELD-shape (S=128, 5 turns), B=32/GPU"),
}
MODELS = {"small": dict(n_embd=768, n_layer=12, n_head=12), "medium": dict(n_embd=1024, n_layer=24, n_head=16)}


def pmc_mfma_busy(key, config: str = "c2"):
    """MFMA busy fraction of the probed kernel from the newest committed MFMA PMC pass
    (profiles/r*_pmc_mfma.json, written by tools/pmc_mfma.py: SQ_VALU_MFMA_BUSY_CYCLES over
    GRBM_GUI_ACTIVE/8 x 1024 SIMDs).  None when no summary covers the probe."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r*_pmc_mfma.json")))
    if key is None or config != "c2":
        return None
    for fn in reversed(files):
        with open(fn) as f:
            rec = json.load(f).get(key)
        if rec:
            return round(rec["mfma_busy_pct"] / 100.0, 4)
    return None


def flops_per_utterance(S: int, E: int = 768, L: int = 12, V: int = 50260) -> float:
    """3·S·[L·(28E² + 4E²·Sc/S + 2SE + 4ScE) + 2EV] with Sc = S (causal self-attention
    counted at S²/2, cross-attention in full; LN/softmax/CE/AdamW/embedding excluded)."""
    Sc = S
    f_tok = L * (28 * E * E + 4 * E * E * Sc / S + 2 * S * E + 4 * Sc * E) + 2 * E * V
    return 3.0 * S * f_tok


def cpu_baseline(S, turns, B, model="small", feat_dim=768, seconds_target=20.0):
    """Time the CPU oracle (fp32) doing the same train step on a bounded sample."""
    from oracle import gpt2_oracle as O
    from ergm_amd.data import synthetic_batch
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    torch.set_num_threads(n)
    cfg = O.OracleConfig(**MODELS[model], feat_dim=feat_dim)
    P = O.init_params(cfg, seed=0, perturb=False)
    st = O.AdamWState()
    batch = synthetic_batch(B, S, n_turns=turns, seed=123, feat_dim=feat_dim)
    lr = 2e-5
    _, g = O.loss_and_grads(P, cfg, batch)  # warm-up step
    O.adamw_step(P, g, st, lr)
    steps, t0 = 0, time.perf_counter()
    while True:
        _, g = O.loss_and_grads(P, cfg, batch)
        O.adamw_step(P, g, st, lr)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds_target or steps >= 3:
            break
    return {"value": round(B * steps / el, 4), "unit": "utterances/s", "cores": n, "kind": "port",
            "sample": f"{steps} full fp32 train steps (fwd+bwd+AdamW) of the CPU oracle at B={B}, S={S}, "
                      f"GPT-2-{model}+fusion, after 1 warm-up step; torch CPU threads={n}"}


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """``--gpus N`` without an external launcher: start N fresh rank processes of this script (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their environment)
    and return the first non-zero exit status.  The parent never touches the GPU (no HIP call before
    the children exist); rank 0's stdout carries the JSON line.  A failing rank ends the others."""
    import subprocess
    env0 = dict(os.environ)
    env0.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    port = env0.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, ERGM_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:  # exact PIDs this launcher started
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-overlap-optim", action="store_true",
                    help="apply AdamW in opt.step() instead of per gradient bucket during backward")
    ap.add_argument("--adamw-blocks", type=int, default=None,
                    help="grid cap of the overlapped per-bucket AdamW (default: FusedAdamW.overlap_blocks)")
    ap.add_argument("--probe", type=int, default=5,
                    help="roofline probe: 5 = every weight-gradient GEMM launch (the dominant time class, default); "
                         "1 = LM-head forward main launch, 2 = LM-head dX, 3 = LM-head dW, 4 = caption K/V GEMM")
    ap.add_argument("--no-fp8", action="store_true", help="c5: run the forward GEMMs in bf16 instead of fp8")
    ap.add_argument("--torch-metrics", action="store_true",
                    help="per-step metrics with framework ops instead of the executor's loss finalisation")
    ap.add_argument("--backend", default=None, help="torch.distributed backend for N > 1 (default nccl = RCCL)")
    ap.add_argument("--defer-update", action="store_true",
                    help="single process: run the block updates after the backward, overlapping the next forward")
    ap.add_argument("--no-gpu-only", dest="gpu_only", action="store_false",
                    help="skip the extra K steps enqueued behind a spin kernel (no host in the loop) that give "
                         "gpu_only_ms_per_step")
    ap.add_argument("--pdrop", type=float, default=None,
                    help="attn/resid/embd dropout (default: the config's 0.1, as the reference trains; 0 = off)")
    ap.add_argument("--seed", type=int, default=0, help="torch.manual_seed before the model is built (dropout masks)")
    args = ap.parse_args()
    # every ERGM_* variable of this run is recorded in the JSON line (none changes results except the documented
    # data-parallel exchange choices); the library has no knock-out switches, refuse a stale one
    if "ERGM_DIAG_SKIP" in os.environ:
        raise SystemExit("ERGM_DIAG_SKIP is not a switch of this library any more: unset it")
    env_overrides = {k: v for k, v in sorted(os.environ.items()) if k.startswith("ERGM_") and k != "ERGM_BENCH_CHILD"}
    # the data-parallel exchange: the library defaults (fp32 all-reduce = the reference's arithmetic, replicated
    # update) unless the caller opts into the bf16 exchange / sharded update (verdict r05 #7); recorded in `config`
    os.environ.setdefault("ERGM_DP_GRAD", "fp32")
    os.environ.setdefault("ERGM_DP_ZERO", "0")

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # self-launch: one fresh process per GPU, before anything here initialises HIP
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one process per GPU")
    if os.environ.get("ERGM_BENCH_LAUNCH_PROBE") == "1":
        # CPU test hook (tests/test_bench_launch.py): the ranks rendezvous over gloo and report, no GPU
        import torch.distributed as dist
        dist.init_process_group("gloo")
        t = torch.tensor([float(rank)])
        dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"world_size": dist.get_world_size(), "rank_sum": t.item(),
                              "local_ranks": os.environ.get("LOCAL_RANK")}), flush=True)
        dist.destroy_process_group()
        return
    # rehearsal hook (one-GPU box): ERGM_BENCH_REHEARSE=1 puts every rank on cuda:0 and uses gloo (RCCL
    # refuses two ranks on one device), so the data-parallel path of this script runs end to end
    # without a GPU per rank (numbers not meaningful)
    rehearse = os.environ.get("ERGM_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    backend = None
    # host-cost hook (one-GPU box): ERGM_BENCH_FAKE_PG=N runs ONE process as rank 0 of a torch "fake" process
    # group of N ranks, whose collectives do nothing — the whole data-parallel schedule (per-bucket casts,
    # chunk sums, sharded AdamW, master sync) is enqueued and run on the GPU, only the wire is missing, so the
    # step's host enqueue and GPU time under DP can be measured (results and utterances/s not meaningful)
    fake_world = int(os.environ.get("ERGM_BENCH_FAKE_PG", "0"))
    if fake_world > 1 and world == 1:
        import torch.distributed as dist
        from torch.testing._internal.distributed.fake_pg import FakeStore
        dist.init_process_group("fake", rank=0, world_size=fake_world, store=FakeStore())
        pg, backend, world = dist.group.WORLD, "fake", fake_world
        args.gpus = fake_world
    if world > 1 and pg is None:
        import torch.distributed as dist
        backend = args.backend or ("gloo" if rehearse else "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        pg = dist.group.WORLD
        got = dist.get_world_size()
        if got != args.gpus:
            raise SystemExit(f"rank {rank}: process group has {got} ranks, --gpus {args.gpus}")

    from ergm_amd import _lib
    from ergm_amd.config import ERGMConfig
    from ergm_amd.data import synthetic_batch
    from ergm_amd.model import GPT2LMHeadModel
    from ergm_amd.optim import FusedAdamW, get_polynomial_decay_schedule_with_warmup

    mname, S, turns, B, Fd, fp8, desc = CONFIGS[args.config]
    fp8 = fp8 and not args.no_fp8
    if not fp8:
        desc = desc.replace("fp8 (e4m3) forward Conv1D GEMMs", "bf16 GEMMs")
    cfg = ERGMConfig(**MODELS[mname], feat_dim=Fd, fp8=fp8)
    if args.pdrop is not None:
        cfg.attn_pdrop = cfg.resid_pdrop = cfg.embd_pdrop = args.pdrop
    torch.manual_seed(args.seed)  # the dropout mask stream (GPT2LMHeadModel draws its seed from torch's generator)
    model = GPT2LMHeadModel(cfg, device=dev, process_group=pg)
    model.init_weights(seed=0)
    defer = args.defer_update and world == 1
    opt = FusedAdamW([model.flat], lr=2e-5, model=model, overlap=not args.no_overlap_optim, defer=defer)
    if args.adamw_blocks is not None:
        opt.overlap_blocks = args.adamw_blocks
    total = args.warmup + args.steps
    sched = get_polynomial_decay_schedule_with_warmup(opt, num_warmup_steps=int(0.1 * total),
                                                      num_training_steps=total, power=2)
    big_feat = args.config == "c4"  # "larger audio/visual feat" (pooling is build-side)
    batch = synthetic_batch(B, S, n_turns=turns, seed=1000 + rank, feat_dim=Fd, visual_rows=197 if big_feat else 1)
    kw = dict(input_ids=batch["input_ids"], token_type_ids=batch["token_type_ids"], labels=batch["labels"],
              emotion_labels=batch["emotion_labels"], caption_ids=batch["caption_ids"], imgs=batch["visual_feat"],
              auds=batch["audio_feat"])
    kw = {k: v.to(dev) for k, v in kw.items()}  # inputs resident in HBM before timing
    aud_hidden = None
    if big_feat:  # wav2vec2-shaped encoder output, pooled inside every timed step
        from ergm_amd.ops import feat_pool
        aud_hidden = (0.1 * torch.randn(B, 400, Fd, generator=torch.Generator().manual_seed(7 + rank))).to(dev)
    loss_acc = torch.zeros(2, device=dev)
    correct = torch.zeros(1, device=dev, dtype=torch.int64)
    # the trainer's per-step metrics (src/main.py:158-169), kept on device (no host sync) and accumulated by
    # the executor's loss finalisation (--torch-metrics: the equivalent framework ops after each step)
    if not args.torch_metrics:
        model.set_train_metrics(loss_acc, correct)

    def step():
        if aud_hidden is not None:
            kw["auds"] = feat_pool(aud_hidden)
        out = model(**kw)
        opt.zero_grad()
        out.loss.backward()
        opt.step()
        sched.step()
        if args.torch_metrics:
            loss_acc[0] += out.loss.detach()
            loss_acc[1] += out.loss_lm
            correct.add_((out.emotion_logits.argmax(-1) == kw["emotion_labels"]).sum())
        return out

    for _ in range(args.warmup):
        step()
    runner = next(iter(model._runners.values()))
    lib = _lib.load()
    import ctypes as C
    # roofline probe: event pairs around every weight-gradient GEMM launch (the dominant time class:
    # ergm_model_set_probe_list) in extra steps right after the timed region (a timing event per launch
    # slows the step ~10 %, so the timed steps run unprobed), or one pair around the --probe launch inside
    # every timed step
    NPR = 4 * cfg.n_layer * 3 + 8
    n_probe_steps = min(args.steps, 10)
    if args.probe == 5:
        plist = []
        for _ in range(n_probe_steps):
            b, e = [_lib.HipEvent() for _ in range(NPR)], [_lib.HipEvent() for _ in range(NPR)]
            plist.append((b, e, (C.c_void_p * NPR)(*[x.ev.value for x in b]),
                          (C.c_void_p * NPR)(*[x.ev.value for x in e]), (C.c_double * NPR)()))
    evs = [(_lib.HipEvent(), _lib.HipEvent()) for _ in range(args.steps)]
    counts = []

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    sync0 = sum(r.host_sync_s for r in model._runners.values())
    prof = None
    prof_bwd = None
    if os.environ.get("ERGM_BENCH_CPROFILE"):  # host-cost diagnostics: cProfile of the timed loop only
        import cProfile
        from ergm_amd import runtime as _rt
        prof = cProfile.Profile()
        # the backward (native stages + the data-parallel exchange) runs on autograd's device thread, which the
        # main thread's profiler does not see: a second profiler inside ModelRunner.backward
        prof_bwd = cProfile.Profile()
        _bwd = _rt.ModelRunner.backward

        def _prof_backward(self, *a, **k):
            prof_bwd.enable()
            try:
                return _bwd(self, *a, **k)
            finally:
                prof_bwd.disable()
        _rt.ModelRunner.backward = _prof_backward
        prof.enable()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if args.probe != 5:
            e0, e1 = evs[i]
            _lib.check(lib.ergm_model_set_probe(runner.plan, args.probe, e0.ev, e1.ev), "ergm_model_set_probe")
        step()
    t_enq = time.perf_counter() - t0  # host time to enqueue the K steps (≈ dt when host-bound)
    if prof is not None:
        prof.disable()
        prof.dump_stats(os.environ["ERGM_BENCH_CPROFILE"])
        prof_bwd.dump_stats(os.environ["ERGM_BENCH_CPROFILE"] + ".bwd")
        _rt.ModelRunner.backward = _bwd
    t_sync = sum(r.host_sync_s for r in model._runners.values()) - sync0  # of it: waiting (DP row count)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    lib.ergm_model_set_probe(runner.plan, 0, None, None)
    metrics = (loss_acc[0].item(), correct.item())  # before any untimed extra step
    # host cost of one step: a few steps enqueued while a spin kernel keeps the device busy, so no launch
    # waits for queue space (in the timed loop the host runs ahead until the queue is full, and from then
    # on its enqueue time is the device's step time)
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2.4e9 * 0.15))
    th = time.perf_counter()
    for _ in range(3):
        step()
    host_ms = round(1000.0 * (time.perf_counter() - th) / 3, 3)
    torch.cuda.synchronize()
    if args.probe == 5:
        tp = time.perf_counter()
        for pb in plist:
            _lib.check(lib.ergm_model_set_probe_list(runner.plan, 5, pb[2], pb[3], pb[4], NPR), "ergm_model_set_probe_list")
            step()
            counts.append(lib.ergm_model_probe_count(runner.plan))
        lib.ergm_model_set_probe(runner.plan, 0, None, None)
        torch.cuda.synchronize()
        probe_step_ms = 1000.0 * (time.perf_counter() - tp) / len(plist)
        # per launch: algorithmic FLOPs recorded by the executor, duration from the event pair
        durs, flops = [], []
        for (b, e, _, _, fl), n in zip(plist, counts):
            durs += [b[k].elapsed_ms(e[k]) for k in range(n)]
            flops += [fl[k] for k in range(n)]
        if os.environ.get("ERGM_BENCH_PHASES"):  # diagnostics: device time of forward / backward per step
            ph = []
            for _ in range(5):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record()
                out = model(**kw)
                ev[1].record()
                opt.zero_grad()
                out.loss.backward()
                opt.step()
                sched.step()
                ev[2].record()
                ph.append(ev)
            torch.cuda.synchronize()
            res = {"forward_ms": sum(e[0].elapsed_time(e[1]) for e in ph) / len(ph),
                   "backward_opt_ms": sum(e[1].elapsed_time(e[2]) for e in ph) / len(ph),
                   "step_ms": sum(e[0].elapsed_time(e[2]) for e in ph) / len(ph)}
            with open(os.environ["ERGM_BENCH_PHASES"], "w") as f:
                json.dump(res, f)
        if os.environ.get("ERGM_BENCH_FWD_DETAIL"):  # the same for the block forward GEMMs (list probe 6)
            NF = 6 * 2 * cfg.n_layer + 8
            fl = []
            for _ in range(3):
                b, e = [_lib.HipEvent() for _ in range(NF)], [_lib.HipEvent() for _ in range(NF)]
                arr = ((C.c_void_p * NF)(*[x.ev.value for x in b]), (C.c_void_p * NF)(*[x.ev.value for x in e]),
                       (C.c_double * NF)())
                _lib.check(lib.ergm_model_set_probe_list(runner.plan, 6, arr[0], arr[1], arr[2], NF), "probe list")
                step()
                fl.append((b, e, arr[2], lib.ergm_model_probe_count(runner.plan)))
            lib.ergm_model_set_probe(runner.plan, 0, None, None)
            n = min(x[3] for x in fl)
            det = [{"k": k, "gflop": fl[0][2][k] / 1e9,
                    "us": 1000.0 * sum(x[0][k].elapsed_ms(x[1][k]) for x in fl) / len(fl)} for k in range(n)]
            with open(os.environ["ERGM_BENCH_FWD_DETAIL"], "w") as f:
                json.dump(det, f, indent=0)
        if os.environ.get("ERGM_BENCH_DW_DETAIL"):  # per launch position: mean in-step duration and FLOPs
            n = min(counts)
            det = [{"k": k, "gflop": plist[0][4][k] / 1e9,
                    "us": 1000.0 * sum(pb[0][k].elapsed_ms(pb[1][k]) for pb in plist) / len(plist)} for k in range(n)]
            with open(os.environ["ERGM_BENCH_DW_DETAIL"], "w") as f:
                json.dump(det, f, indent=0)
        # secondary: the LM head's main forward launch, timed in extra (untimed) steps after the timed region
        lm = []
        for _ in range(3):
            e0, e1 = _lib.HipEvent(), _lib.HipEvent()
            _lib.check(lib.ergm_model_set_probe(runner.plan, 1, e0.ev, e1.ev), "ergm_model_set_probe")
            step()
            lm.append((e0, e1))
        lib.ergm_model_set_probe(runner.plan, 0, None, None)
        lm_ms = sum(a.elapsed_ms(b) for a, b in lm) / len(lm)
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    if args.probe != 5:
        probe_ms = sum(a.elapsed_ms(b) for a, b in evs) / len(evs)
    utt = B * world * args.steps
    value = utt / dt
    ms_step = 1000.0 * dt / args.steps
    T = B * S
    V, E = cfg.vocab_size, cfg.n_embd
    Vp = model.layout.vocab_pad
    n0 = min(V, lmhead_split_cols(T, Vp))
    lm_name = (f"LM-head forward main GEMM [T,E]x[E,{n0}] (pipelined MFMA GEMM, 256x256 tiles in whole rounds of "
               f"256 CUs, bf16 out; the last {Vp - n0} vocabulary columns run as a separate small-tile launch)"
               if n0 < V else "LM-head forward GEMM [T,E]x[E,V] (pipelined MFMA GEMM, bf16 out)")
    lm_flops = 2.0 * T * n0 * E
    if args.probe == 5:
        n_l = len(durs) // max(1, len(counts))
        probe_ms = sum(durs) / len(durs)
        probe_flops = sum(flops) / len(flops)
        achieved = sum(flops) / (sum(durs) * 1e-3) / 1e12
        probe_name = (f"weight-gradient GEMM class (dW = X^T.dY, KM x KN operands, fp32 out; the step's largest "
                      f"time class): {n_l} launches per step for every block's 6 Conv1D dW (bias gradient summed in the same "
                      "GEMM; pairs whose problems underfill the chip grouped into one launch), the stacked caption K/V dW and "
                      "the tied LM-head dW; achieved = sum of their algorithmic FLOPs "
                      f"/ sum of their in-step launch durations (HIP events around each launch, {n_probe_steps} steps run "
                      "right after the timed region)")
        traffic, traffic_src = pmc_traffic("dw_class", args.config)
        mfma_busy = pmc_mfma_busy("dw_class", args.config)
    else:
        probe_flops = {1: lm_flops, 2: 2.0 * T * V * E, 3: 2.0 * T * V * E,
                       4: 2.0 * T * E * (2 * E * cfg.n_layer)}[args.probe]
        probe_name = {1: lm_name, 2: "LM-head dX GEMM", 3: "LM-head dW GEMM", 4: "stacked caption K/V GEMM"}[args.probe]
        achieved = probe_flops / (probe_ms * 1e-3) / 1e12
        traffic, traffic_src = pmc_traffic("lm_head_fwd" if args.probe == 1 else None, args.config)
        mfma_busy = pmc_mfma_busy("lm_head_fwd" if args.probe == 1 else None, args.config)
    Lyr = cfg.n_layer
    step_flops = flops_per_utterance(S, E, Lyr, V) * B
    rec = {
        "metric": "utterances/sec training, MELD-shape synthetic batch, 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "utterances/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp8e4m3 fwd GEMMs + bf16" if fp8 else "bf16",
        "dropout": {"attn": cfg.attn_pdrop, "resid": cfg.resid_pdrop, "embd": cfg.embd_pdrop, "mode": "train"},
        "data": f"synthetic (seeded MELD-shape token/feature batches; random-init GPT-2-{mname} weights)",
        "config": {"workload": desc, "model": f"GPT-2-{mname} (L={Lyr}, E={E}, H={cfg.n_head}, V={V}) + "
                   "cross-attention caption fusion + emotion head", "global_batch": B * world, "seq_len": S,
                   "parallelism": f"dp{world}",
                   "dp_grad_exchange": os.environ["ERGM_DP_GRAD"] + (" (narrower than the reference's fp32 sum)"
                                                                      if os.environ["ERGM_DP_GRAD"] == "bf16" else ""),
                   "dp_sharded_optimizer": os.environ["ERGM_DP_ZERO"] == "1"},
        "roofline": {"bound": "mfma", "kernel": probe_name, "achieved": round(achieved, 1),
                     "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                     "traffic": traffic, "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": traffic_src,
                     "mfma_busy_pmc": mfma_busy,
                     "avg_launch_ms": round(probe_ms, 4),
                     "flops_per_launch": probe_flops,
                     "probe_steps_ms_per_step": round(probe_step_ms, 3) if args.probe == 5 else None},
        "roofline_secondary": ({"kernel": lm_name, "flops_per_launch": lm_flops, "avg_launch_ms": round(lm_ms, 4),
                                "achieved": round(lm_flops / (lm_ms * 1e-3) / 1e12, 1),
                                "frac": round(lm_flops / (lm_ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
                                "traffic": pmc_traffic("lm_head_fwd", args.config)[0],
                                "timed": "3 extra steps after the timed region"} if args.probe == 5 else None),
        "mfma_step": {"flops_per_step": step_flops, "achieved_tflops": round(step_flops / (ms_step * 1e-3) / 1e12, 1),
                      "frac": round(step_flops / (ms_step * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
                      "ceiling_utt_per_s_per_gpu": round(PEAK_BF16_TFLOPS * 1e12 / flops_per_utterance(S, E, Lyr, V),
                                                         0)},
        "optimizer": "FusedAdamW " + ((f"per-bucket, overlapped with backward (grid cap {opt.overlap_blocks}), "
                                       + ("scheduled by the native executor" if world == 1 else
                                          "after each bucket's exchange (comm stream)"))
                                      if not args.no_overlap_optim else "after backward"),
        "env": env_overrides,
        "world_size": world,
        "dp": {"backend": backend, "rehearsal": rehearse, "grad_comm": runner.dp.grad_comm,
               "grad_bytes_sent_per_rank_per_step": runner.dp.bytes_per_step,
               "exchange": ("bf16 all-to-all + fp32 chunk sum (reduce-scatter), then " +
                            ("AdamW on this rank's chunk + bf16 all-gather of the updated shadow (ZeRO-1)"
                             if runner.dp.zero else "bf16 all-gather of the reduced gradient")
                            if runner.dp.grad_comm == "bf16" else "fp32 all-reduce"),
               "sharded_optimizer": runner.dp.zero} if world > 1 else None,
        "host_enqueue_ms_per_step": host_ms,
        "host_enqueue_ms_per_step_in_timed_loop": round(1000.0 * t_enq / args.steps, 3),
        # under DP the host also blocks once per step on the compact lookup's row count: the rest is host work
        "host_busy_ms_per_step_in_timed_loop": round(1000.0 * (t_enq - t_sync) / args.steps, 3),
        "train_metrics": {"mean_loss": round(metrics[0] / total, 4),
                          "emotion_acc": round(metrics[1] / (B * total), 4)},
    }
    if args.gpu_only and world == 1:
        # the same K steps enqueued while the GPU spins: the host is never on the critical path
        torch.cuda.synchronize()
        g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2.4e9 * (0.05 + 0.006 * args.steps)))
        g0.record()
        for i in range(args.steps):
            step()
        g1.record()
        torch.cuda.synchronize()
        rec["gpu_only_ms_per_step"] = round(g0.elapsed_time(g1) / args.steps, 3)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(S, turns, B, mname, Fd)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
