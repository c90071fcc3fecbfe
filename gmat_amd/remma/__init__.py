from gmat_amd.remma.annotation import annotation_snp_pos
from gmat_amd.remma.random_pair import random_pair, random_pairAD
from gmat_amd.remma.remma_epiAA.remma_epiAA import remma_epiAA, remma_epiAA_parallel
from gmat_amd.remma.remma_epiAA.remma_epiAA_pair import remma_epiAA_pair
from gmat_amd.remma.remma_epiAA.remma_epiAA import _remma_epiAA, _remma_epiAA_parallel
from gmat_amd.remma.remma_epiAA.remma_epiAA_pair import _remma_epiAA_pair
from gmat_amd.remma.remma_epiAD.remma_epiAD import remma_epiAD, remma_epiAD_parallel, _remma_epiAD
from gmat_amd.remma.remma_epiAD.remma_epiAD_pair import remma_epiAD_pair, _remma_epiAD_pair
from gmat_amd.remma.remma_epiDD.remma_epiDD import remma_epiDD, remma_epiDD_parallel, _remma_epiDD
from gmat_amd.remma.remma_epiDD.remma_epiDD_pair import remma_epiDD_pair, _remma_epiDD_pair
from gmat_amd.remma.remma_add import remma_add, _remma_add
from gmat_amd.remma.remma_dom import remma_dom, _remma_dom

import sys as _sys
import types as _types


class _RemmaModule(_types.ModuleType):
    """Keeps the exported functions remma_epiAA / remma_epiAD / remma_epiDD when their same-named
    subpackages are imported again through the ``gmat`` alias (``from gmat.remma.remma_epiAA import
    remma_epiAA``): the import system then sets the parent's attribute to the subpackage, and a later
    ``gmat_amd.remma.remma_epiAA(...)`` found a module instead of the function."""

    def __setattr__(self, name, value):
        cur = self.__dict__.get(name)
        if isinstance(value, _types.ModuleType) and callable(cur) and not isinstance(cur, _types.ModuleType):
            return
        super().__setattr__(name, value)


_sys.modules[__name__].__class__ = _RemmaModule
