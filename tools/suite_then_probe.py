"""Long-process resume probe (GPU box): run the GPU test suite in this process (pytest.main, the trainer test
deselected), then tools/race_probe.py's perturbed resume runs in the same process, so the probe sees the state
≈ 280 earlier tests leave behind (allocator pools, streams and HIP queues created and destroyed, plans cached).
Usage: python tools/suite_then_probe.py [reps_per_mode]"""
import os
import sys

import pytest

here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(here, "tools"))

if __name__ == "__main__":  # the dist tests spawn children, which import this module
    files = os.environ.get("SUITE", "tests").split()  # a subset of the suite (bisection), default all of it
    rc = pytest.main(["-x", "-q", "-m", "gpu", "-p", "no:cacheprovider", *files,
                      "--deselect", "tests/test_gpu_train.py::test_trainer_epochs_checkpoint_and_resume"])
    print(f"suite rc {int(rc)}", flush=True)
    import race_probe  # noqa: E402

    R = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    bad = race_probe.main(R) if R > 0 else 0
    # the trainer test itself, repeated in this process (its models stay alive across its three runs, as in the suite)
    import torch
    from test_gpu_train import test_trainer_epochs_checkpoint_and_resume as resume_test
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    fails = 0
    for i in range(n):
        try:
            resume_test(torch.device("cuda:0"))
        except AssertionError as ex:
            fails += 1
            print(f"trainer test repetition {i}: FAILED {str(ex)[:400]}", flush=True)
    print(f"trainer test: {n - fails}/{n} passed", flush=True)
    sys.exit(1 if bad or fails else int(rc))
