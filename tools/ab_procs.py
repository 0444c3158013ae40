"""A/B of executor variants on the C2 step, one worker PROCESS per variant (each with its own HIP streams and
hardware queues — several models in one process share the process's 4 hardware queues and can serialise each
other's streams, which made tools/ab_inproc.py's third and later variants ~20 % slow).  The controller lets the
workers run blocks of steps in turn (never two at once), so slow box drift hits every variant alike.

CAVEAT: the idle workers keep their hardware queues mapped, and beyond the firmware's queue slots the active
worker is time-sliced against them (an identical second worker measured +4.4 %): prefer tools/ab.sh.
Usage (GPU box): python tools/ab_procs.py "label:ENV=v,ENV2=w" "label2:" [--blocks 8] [--steps 10]
Prints the median ms/step per variant."""
import os
import statistics
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(nsteps: int) -> None:
    sys.path.insert(0, HERE)
    import torch
    import bench
    from ergm_amd.config import ERGMConfig
    from ergm_amd.data import synthetic_batch
    from ergm_amd.model import GPT2LMHeadModel
    from ergm_amd.optim import FusedAdamW, get_polynomial_decay_schedule_with_warmup
    dev = torch.device("cuda:0")
    mname, S, turns, B, Fd, fp8, _ = bench.CONFIGS["c2"]
    cfg = ERGMConfig(**bench.MODELS[mname], feat_dim=Fd, fp8=fp8)
    model = GPT2LMHeadModel(cfg, device=dev)
    model.init_weights(seed=0)
    opt = FusedAdamW([model.flat], lr=2e-5, model=model, overlap=True)
    sched = get_polynomial_decay_schedule_with_warmup(opt, num_warmup_steps=10, num_training_steps=10 ** 6, power=2)
    batch = synthetic_batch(B, S, n_turns=turns, seed=1000, feat_dim=Fd, visual_rows=1)
    kw = dict(input_ids=batch["input_ids"], token_type_ids=batch["token_type_ids"], labels=batch["labels"],
              emotion_labels=batch["emotion_labels"], caption_ids=batch["caption_ids"], imgs=batch["visual_feat"],
              auds=batch["audio_feat"])
    kw = {k: v.to(dev) for k, v in kw.items()}
    acc, hits = torch.zeros(2, device=dev), torch.zeros(1, device=dev, dtype=torch.int64)
    model.set_train_metrics(acc, hits)

    def step():
        out = model(**kw)
        opt.zero_grad()
        out.loss.backward()
        opt.step()
        sched.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    print("ready", flush=True)
    for line in sys.stdin:
        if line.strip() != "go":
            break
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(nsteps):
            step()
        torch.cuda.synchronize()
        print(f"{1000.0 * (time.perf_counter() - t0) / nsteps:.4f}", flush=True)


def main():
    blocks = int(sys.argv[sys.argv.index("--blocks") + 1]) if "--blocks" in sys.argv else 8
    nsteps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 10
    if "--worker" in sys.argv:
        return worker(nsteps)
    specs = [a for i, a in enumerate(sys.argv[1:], 1) if not a.startswith("--") and sys.argv[i - 1] not in
             ("--blocks", "--steps")]
    procs = []
    for spec in specs:
        label, envs = (spec.split(":", 1) + [""])[:2]
        env = dict(os.environ)
        for kv in filter(None, envs.split(",")):
            k, v = kv.split("=", 1)
            env[k] = v
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker", "--steps", str(nsteps)],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env, cwd=HERE)
        procs.append((label, p, []))
    for label, p, _ in procs:
        if p.stdout.readline().strip() != "ready":
            raise SystemExit(f"worker {label} failed to start")
    try:
        for _ in range(blocks):
            for label, p, times in procs:
                p.stdin.write("go\n")
                p.stdin.flush()
                times.append(float(p.stdout.readline()))
    finally:
        for _, p, _ in procs:
            p.stdin.close()
            p.wait(timeout=60)
    base = statistics.median(procs[0][2])
    for label, _, times in procs:
        med = statistics.median(times)
        print(f"{label:12s} median {med:7.3f} ms/step  ({100.0 * (med / base - 1):+5.1f} %)  min {min(times):7.3f}  "
              f"all {' '.join(f'{t:.2f}' for t in times)}", flush=True)


if __name__ == "__main__":
    main()
