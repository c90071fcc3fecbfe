"""gmat_amd -- MI355X-native (gfx950) implementation of GMAT's REMMAX hot path.

Drop-in modules mirroring the reference's import paths:
  gmat_amd.gmatrix  : agmat, dgmat_as, output_mat
  gmat_amd.uvlmm    : wemai_multi_gmat, _wemai_multi_gmat, design_matrix_wemai_multi_gmat
  gmat_amd.remma    : remma_epiAA/AD/DD (+ _parallel, _pair, private forms), annotation_snp_pos,
                      random_pair, random_pairAD
Compute runs in libgmat_hip.so (hand-written HIP kernels; C ABI in include/gmat_hip.h).
"""
__version__ = "0.1.0"

# GMAT_NUM_GPUS=N: this command line runs as N ranks of one job (gmat_amd.launch.spawn_from_env); the
# parent process only starts them and exits with their status, before the script reaches a GPU call
import os as _os

if _os.environ.get("GMAT_NUM_GPUS", "").strip() and _os.environ.get("WORLD_SIZE") is None:
    from . import launch as _launch

    _rc = _launch.spawn_from_env()
    if _rc is not None:
        raise SystemExit(_rc)
