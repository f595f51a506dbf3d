"""Realm punch matcher on the GPU (hyobfs_punch_match_batch, punch_conn.go:146-165):
every datagram against every registered attempt, vs the hashlib restatement."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from oracle import realm_ref as rref  # noqa: E402
from punch_cases import punch_batch  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,m,seed", [(1, 1, 1), (5000, 1, 2), (20000, 6, 3), (3000, 32, 4)])
def test_match_batch_vs_oracle(gpu, n, m, seed):
    import torch
    from hysteria_amd import realm
    pk, atts, metas = punch_batch(n, m, seed)
    buf = np.frombuffer(b"".join(pk) + bytes(16), np.uint8).copy()
    off = np.concatenate([[0], np.cumsum([len(x) for x in pk])[:-1]]).astype(np.uint64)
    ln = np.array([len(x) for x in pk], np.uint32)
    mt = realm.PunchMatcher(metas)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(gpu)  # noqa: E731
    match = torch.full((n,), -7, dtype=torch.int32, device=gpu)
    ty = torch.zeros(n, dtype=torch.uint8, device=gpu)
    pad = torch.zeros(n, dtype=torch.int32, device=gpu)
    mt.match_batch(d(buf), d(off), d(ln), n, match, ty, pad, attempts=d(mt.attempts))
    torch.cuda.synchronize()
    hm, ht, hp = match.cpu().numpy(), ty.cpu().numpy(), pad.cpu().numpy()
    hits = 0
    for i, x in enumerate(pk):
        j, t, pd = rref.match(x, atts)
        assert (int(hm[i]), int(ht[i]) if j >= 0 else 0, int(hp[i])) == (j, t, pd), i
        hits += j >= 0
    assert n == 1 or 0 < hits < n
