"""Genomic relationship matrices (gmat.gmatrix, gmatrix/__init__.py:1)."""
from gmat_amd.gmatrix.gmatrix import agmat, dgmat_as, output_mat, spd_inverse  # noqa: F401
