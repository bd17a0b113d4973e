"""CPU: the rank-local commutator products' helper (distributed._row_diagonal): the diagonal of a row subset of an
operator whose columns keep their global numbering equals the global operator's diagonal on those rows."""
import types

import numpy as np
import scipy.sparse as sp
import torch

from mp_block_preconditioners_amd.distributed import _row_diagonal
from mp_block_preconditioners_amd._lib import MpbpError


def _sub(M, rows):
    S = M[rows].tocsr()
    S.sort_indices()
    return types.SimpleNamespace(row_ptr=torch.from_numpy(S.indptr.astype(np.int32)),
                                 col_idx=torch.from_numpy(S.indices.astype(np.int32)),
                                 val=torch.from_numpy(S.data.astype(np.float64)), shape=S.shape)


def test_row_diagonal_matches_global():
    rng = np.random.default_rng(3)
    n = 200
    M = (sp.random(n, n, density=0.05, random_state=4) + sp.diags(rng.uniform(1, 2, n))).tocsr()
    rows = np.sort(rng.choice(n, 57, replace=False))
    d = _row_diagonal(_sub(M, rows), torch.from_numpy(rows.astype(np.int32)))
    assert np.array_equal(d.numpy(), M.diagonal()[rows])


def test_row_diagonal_missing_entry_raises():
    M = sp.csr_matrix(np.array([[1.0, 2.0], [3.0, 0.0]]))
    M.eliminate_zeros()
    try:
        _row_diagonal(_sub(M, np.array([0, 1])), torch.tensor([0, 1], dtype=torch.int32))
    except MpbpError:
        return
    raise AssertionError("a row without its diagonal entry must raise")
