"""In-process A/B of executor variants on the C2 step: one model per variant (plan-level switches are read
from the environment when each model's plan is created), the variants' steps run in alternating blocks
inside ONE process, so slow box drift (clock, thermals) hits every variant alike.
CAVEAT: every model's executor creates its own streams and a process maps its streams onto 4 hardware queues,
so from the third variant on streams of different models share queues and can serialise each other (~+20 %
whatever the variant): compare two variants at a time, and confirm with sequential runs (tools/ab.sh).

Usage (GPU box): python tools/ab_inproc.py "label:ENV=v,ENV2=w:defer" "label2::" [--blocks 8] [--steps 10]
  the third field holds comma-separated flags: defer (deferred block updates), nb=N (AdamW grid cap),
  ov=M/N/K/a_layout/b_layout/cfg/split (a GEMM configuration override, set before each of the variant's blocks;
  same split as the automatic plan, so the scratch sized at plan creation fits).  Prints the median ms/step per variant."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    blocks = int(sys.argv[sys.argv.index("--blocks") + 1]) if "--blocks" in sys.argv else 8
    nsteps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 10
    args = [a for a in args if not a.isdigit()]
    from ergm_amd.config import ERGMConfig
    from ergm_amd.data import synthetic_batch
    from ergm_amd.model import GPT2LMHeadModel
    from ergm_amd.optim import FusedAdamW, get_polynomial_decay_schedule_with_warmup
    import bench
    dev = torch.device("cuda:0")
    mname, S, turns, B, Fd, fp8, _ = bench.CONFIGS["c2"]
    variants = []
    for spec in args:
        label, envs, flags = (spec.split(":") + ["", ""])[:3]
        saved = {}
        for kv in filter(None, envs.split(",")):
            k, v = kv.split("=", 1)
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        cfg = ERGMConfig(**bench.MODELS[mname], feat_dim=Fd, fp8=fp8)
        model = GPT2LMHeadModel(cfg, device=dev)
        model.init_weights(seed=0)
        opt = FusedAdamW([model.flat], lr=2e-5, model=model, overlap=True, defer="defer" in flags)
        for f in flags.split(","):
            if f.startswith("nb="):  # grid cap of the overlapped AdamW launches
                opt.overlap_blocks = int(f[3:])
        sched = get_polynomial_decay_schedule_with_warmup(opt, num_warmup_steps=10, num_training_steps=10 ** 6,
                                                          power=2)
        batch = synthetic_batch(B, S, n_turns=turns, seed=1000, feat_dim=Fd, visual_rows=1)
        kw = dict(input_ids=batch["input_ids"], token_type_ids=batch["token_type_ids"], labels=batch["labels"],
                  emotion_labels=batch["emotion_labels"], caption_ids=batch["caption_ids"],
                  imgs=batch["visual_feat"], auds=batch["audio_feat"])
        kw = {k: v.to(dev) for k, v in kw.items()}
        acc = torch.zeros(2, device=dev)
        hits = torch.zeros(1, device=dev, dtype=torch.int64)
        model.set_train_metrics(acc, hits)

        def step(model=model, opt=opt, sched=sched, kw=kw):
            out = model(**kw)
            opt.zero_grad()
            out.loss.backward()
            opt.step()
            sched.step()

        for _ in range(3):  # the plan is created (and the environment read) here
            step()
        torch.cuda.synchronize()
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        ovs = [tuple(int(x) for x in f[3:].split("/")) for f in flags.split(",") if f.startswith("ov=")]
        variants.append((label, step, [], ovs))
    from ergm_amd import _lib as L
    lib = L.load()
    all_ov = {o[:5] for v in variants for o in v[3]}

    def use(ovs):  # GEMM configuration overrides of one variant (cfg only: the plans' scratch is unchanged)
        for key in all_ov:
            L.check(lib.ergm_gemm_set_override(*key, -1, 1), "override reset")
        for o in ovs:
            L.check(lib.ergm_gemm_set_override(*o), "override")
    for _ in range(blocks):
        for label, step, times, ovs in variants:
            use(ovs)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(nsteps):
                step()
            torch.cuda.synchronize()
            times.append(1000.0 * (time.perf_counter() - t0) / nsteps)
    base = statistics.median(variants[0][2])
    for label, _, times, _ in variants:
        med = statistics.median(times)
        print(f"{label:12s} median {med:7.3f} ms/step  ({100.0 * (med / base - 1):+5.1f} %)  min {min(times):7.3f}  "
              f"all {' '.join(f'{t:.2f}' for t in times)}", flush=True)


if __name__ == "__main__":
    main()
