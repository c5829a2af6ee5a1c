"""Per-shape GEMM selection for the learner: PyTorch TunableOp over the hipBLASLt and rocBLAS solutions.

The update's GEMMs are few shapes repeated thousands of times (the trunks, the LSTM input projection, the
per-step recurrent product (B, 128) x (128, 512) and its BPTT mirror, the split-K weight gradients), and the
library default is not the fastest solution for the small ones: e.g. the recurrent product at B = 4096 runs
11-13 µs under the default hipBLASLt pick and 9.7 µs under the rocBLAS solution TunableOp picks.  Config D's
update: 21.8-22.4 -> 20.0-20.8 ms (``profiles/r05/learn/tunableop_ab.txt``).

``gemm_tuned_gfx950.csv`` holds the results of a tuning run of ``scripts/bench_learner.py`` on config D
(``scripts/archive/r05_learn_tunable.sh``); TunableOp only uses it when its validators (torch, HIP, hipBLASLt, rocBLAS
versions and the GPU arch) match this process.  Shapes it lacks (other env counts, other minibatch sizes) take
the library's own heuristic pick: no GEMM is timed online by default, so the solution a shape gets does not depend
on a timing run and is the same on every run and every rank.  ``OUZ_TUNABLEOP_TUNE=1`` opts in to online tuning
of the missing shapes; only then are results written (with the shipped ones) to a per-user cache file at exit,
and that file is read back by later runs.  ``OUZ_TUNABLEOP=0`` leaves TunableOp alone; a ``PYTORCH_TUNABLEOP_*``
setting in the environment means the user drives TunableOp and nothing is changed here.  TunableOp is
process-wide: it applies to every GEMM of the process once a training learner is built (inference-only callers,
``play.py``, build their learner with ``tuned_gemms=False``).
"""
import os
import tempfile
import warnings

import torch

SHIPPED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_tuned_gfx950.csv")
_state = {"done": False}


def cache_file():
    return os.environ.get("OUZ_TUNABLEOP_FILE") or os.path.join(
        tempfile.gettempdir(), f"ouzelum_tunableop_{os.getuid()}.csv")


def enable_tuned_gemms(device):
    """Turn TunableOp on for this process with the shipped results preloaded (once).  Returns whether it is on."""
    device = torch.device(device)
    if device.type != "cuda" or os.environ.get("OUZ_TUNABLEOP", "1") == "0":
        return False
    T = torch.cuda.tunable
    if any(k.startswith("PYTORCH_TUNABLEOP_") for k in os.environ):
        return T.is_enabled()
    if _state["done"]:
        return True
    tune = os.environ.get("OUZ_TUNABLEOP_TUNE", "0") == "1"
    T.enable(True)
    T.tuning_enable(tune)   # TunableOp writes its results file at exit only while tuning is enabled
    T.set_filename(cache_file(), insert_device_ordinal=True)
    for path in ((SHIPPED, T.get_filename()) if tune else (SHIPPED,)):
        if os.path.exists(path):
            try:
                T.read_file(path)
            except Exception as e:        # another build's or a half-written file: those shapes are tuned instead
                warnings.warn(f"TunableOp results {path} not used: {e}", stacklevel=2)
    _state["done"] = True
    return True
