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
    rc = pytest.main(["-x", "-q", "-m", "gpu", "-p", "no:cacheprovider", os.path.join(here, "tests"),
                      "--deselect", "tests/test_gpu_train.py::test_trainer_epochs_checkpoint_and_resume"])
    print(f"suite rc {int(rc)}", flush=True)
    import race_probe  # noqa: E402

    bad = race_probe.main(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
    sys.exit(1 if bad else int(rc))
