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
