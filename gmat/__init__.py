"""``gmat`` -- the reference's import paths, served by gmat_amd (MI355X / gfx950).

The README and example scripts of the reference import ``gmat.gmatrix``,
``gmat.uvlmm.uvlmm_varcom``, ``gmat.remma.remma_epiAA`` and so on (README.md:98-101,
136-138, 156).  gmat_amd keeps the reference's package layout module for module, so this
package only installs an import hook: every ``gmat.<path>`` resolves to the module object
``gmat_amd.<path>`` itself (one module object per path -- no duplicated state, and
``gmat.remma.remma_epiAA is gmat_amd.remma.remma_epiAA``).  Scripts run unchanged:

    from gmat.gmatrix import agmat
    from gmat.uvlmm.uvlmm_varcom import wemai_multi_gmat
    from gmat.remma.remma_epiAA import remma_epiAA
    from gmat.remma import annotation_snp_pos
"""
import importlib
import importlib.abc
import importlib.util
import sys

_PREFIX = __name__ + "."
_TARGET = "gmat_amd"


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target):
        self._target = target

    def create_module(self, spec):
        mod = importlib.import_module(self._target)
        self._real_spec = getattr(mod, "__spec__", None)
        return mod

    def exec_module(self, module):
        # the target module is already executed; the import system has just pointed its
        # __spec__ at the alias spec: give it back its own
        module.__spec__ = self._real_spec


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith(_PREFIX):
            return None
        real = _TARGET + fullname[len(__name__):]
        if importlib.util.find_spec(real) is None:
            return None
        mod = importlib.import_module(real)
        return importlib.util.spec_from_loader(fullname, _AliasLoader(real),
                                               is_package=hasattr(mod, "__path__"))


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())

from gmat_amd import *  # noqa: E402,F401,F403
