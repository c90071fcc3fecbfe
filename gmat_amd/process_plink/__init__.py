"""PLINK input (gmat.process_plink, process_plink/__init__.py:1-2)."""
from gmat_amd.process_plink.process_plink import read_plink, impute_geno  # noqa: F401
