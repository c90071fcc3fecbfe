"""gmat_amd -- MI355X-native (gfx950) implementation of GMAT's REMMAX hot path.

Drop-in modules mirroring the reference's import paths:
  gmat_amd.gmatrix  : agmat, dgmat_as, output_mat
  gmat_amd.uvlmm    : wemai_multi_gmat, _wemai_multi_gmat, design_matrix_wemai_multi_gmat
  gmat_amd.remma    : remma_epiAA/AD/DD (+ _parallel, _pair, private forms), annotation_snp_pos,
                      random_pair, random_pairAD
Compute runs in libgmat_hip.so (hand-written HIP kernels; C ABI in include/gmat_hip.h).
"""
__version__ = "0.1.0"
