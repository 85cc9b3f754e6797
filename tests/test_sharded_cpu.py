"""Multi-process (gloo, CPU) test of the column-sharded sweep decomposition used at N > 1.

Each rank holds a column shard of X; per sweep there are two sum all-reduces
(S_alpha + X beta, then the partial Gram X_k D_k X_k' + X_k u_k).  Variates are indexed by
the GLOBAL column, so the sharded sweep must reproduce the unsharded one (up to the
summation order of the Gram).  The HIP engine follows the same decomposition with RCCL
(bb_engine.cpp: pre_and_scalars / sweep).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import gibbs
from tests.conftest import synthetic_problem


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, p, sweeps, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, y, btrue = synthetic_problem(n, p, seed=5)
    per = (p + world - 1) // world
    j0, j1 = rank * per, min(p, (rank + 1) * per)
    Xk = np.asfortranarray(X[:, j0:j1])

    def allreduce(v):
        t = torch.from_numpy(np.ascontiguousarray(v))
        dist.all_reduce(t)
        return t.numpy()

    hyper = dict(nu_shape=2.0, nu_rate=2.0, sig2_shape=0.0, sig2_scale=0.0)
    beta_k = btrue[j0:j1] + 0.1
    tau, sig2 = 1.0, 1.0
    hist = []
    for t in range(1, sweeps + 1):
        beta_k, lam_k, tau, sig2 = gibbs.woodbury_sweep_sharded(
            Xk, y, beta_k, j0, p, 0.5, tau, sig2, t, 11, 0, allreduce, hyper)
        full = [torch.zeros(per, dtype=torch.float64) for _ in range(world)]
        pad = np.zeros(per)
        pad[:j1 - j0] = beta_k
        dist.all_gather(full, torch.from_numpy(pad))
        hist.append((np.concatenate([f.numpy() for f in full])[:p], tau, sig2))
    if rank == 0:
        np.savez(out_path, beta=np.array([h[0] for h in hist]), tau=[h[1] for h in hist],
                 sig2=[h[2] for h in hist])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_sweep_matches_unsharded(tmp_path, world):
    n, p, sweeps = 40, 150, 6
    out = str(tmp_path / "sharded.npz")
    mp.spawn(_worker, args=(world, _free_port(), n, p, sweeps, out), nprocs=world, join=True)
    got = np.load(out)
    X, y, btrue = synthetic_problem(n, p, seed=5)

    def ident(v):
        return v

    hyper = dict(nu_shape=2.0, nu_rate=2.0, sig2_shape=0.0, sig2_scale=0.0)
    beta, tau, sig2 = btrue + 0.1, 1.0, 1.0
    for t in range(1, sweeps + 1):
        beta, lam, tau, sig2 = gibbs.woodbury_sweep_sharded(
            np.asfortranarray(X), y, beta, 0, p, 0.5, tau, sig2, t, 11, 0, ident, hyper)
        np.testing.assert_allclose(got["tau"][t - 1], tau, rtol=1e-10)
        np.testing.assert_allclose(got["sig2"][t - 1], sig2, rtol=1e-10)
        d = np.linalg.norm(got["beta"][t - 1] - beta) / np.linalg.norm(beta)
        assert d < 1e-9, (t, d)


def test_sharded_sweep_equals_dense_woodbury_step():
    """world = 1 decomposition == the oracle's beta_step_woodbury with the same variates."""
    import oracle

    X, y, btrue = synthetic_problem(30, 80, seed=2)
    beta = btrue + 0.05
    hyper = dict(nu_shape=2.0, nu_rate=2.0, sig2_shape=0.0, sig2_scale=0.0)
    b1, lam, tau, sig2 = gibbs.woodbury_sweep_sharded(np.asfortranarray(X), y, beta, 0, 80, 0.5,
                                                      1.0, 1.0, 3, 7, 0, lambda v: v, hyper)
    z = oracle.normals(80, 7, 0, 3, oracle.KIND_BETA_Z)
    d = oracle.normals(30, 7, 0, 3, oracle.KIND_DELTA)
    b2 = gibbs.beta_step_woodbury(X, y, lam, sig2, tau, z, d)
    np.testing.assert_allclose(b1, b2, rtol=1e-11, atol=1e-13)


def _nid_worker(rank, world, port, n, p, sweeps, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, y, _ = synthetic_problem(n, p, seed=6)
    per = (p + world - 1) // world
    j0, j1 = rank * per, min(p, (rank + 1) * per)
    Xk = np.asfortranarray(X[:, j0:j1])
    lam_k = 1.02 * np.linalg.eigvalsh(Xk @ Xk.T)[-1]

    def allreduce(v):
        t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64))
        dist.all_reduce(t)
        return t.numpy()

    hyper = dict(nu_shape=2.0, nu_rate=2.0, sig2_shape=0.0, sig2_scale=0.0)
    beta_k = np.full(j1 - j0, 1e-4)
    tau, sig2 = 1e-3, 1.0
    hist, info = [], []
    for t in range(1, sweeps + 1):
        beta_k, _, tau, sig2 = gibbs.woodbury_sweep_sharded(
            Xk, y, beta_k, j0, p, 0.5, tau, sig2, t, 11, 0, allreduce, hyper, know_tau=True,
            nid_lam=lam_k, info=info)
        full = [torch.zeros(per, dtype=torch.float64) for _ in range(world)]
        pad = np.zeros(per)
        pad[:j1 - j0] = beta_k
        dist.all_gather(full, torch.from_numpy(pad))
        hist.append(np.concatenate([f.numpy() for f in full])[:p])
    if rank == 0:
        np.savez(out_path, beta=np.array(hist), K=np.array([k for _, k in info]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_near_identity_matches_unsharded(tmp_path, world):
    """The shards' near-identity solve (the exchanged bound sums decide the path; one exchange
    of X_k u_k and one per product E d) against the unsharded Cholesky draw, from a
    near-null state (tau = 1e-3 known): every sweep takes the Chebyshev path."""
    n, p, sweeps = 40, 150, 4
    out = str(tmp_path / "nid.npz")
    mp.spawn(_nid_worker, args=(world, _free_port(), n, p, sweeps, out), nprocs=world, join=True)
    got = np.load(out)
    assert np.all(got["K"] > 0), got["K"]
    X, y, _ = synthetic_problem(n, p, seed=6)
    hyper = dict(nu_shape=2.0, nu_rate=2.0, sig2_shape=0.0, sig2_scale=0.0)
    beta, tau, sig2 = np.full(p, 1e-4), 1e-3, 1.0
    for t in range(1, sweeps + 1):
        beta, _, tau, sig2 = gibbs.woodbury_sweep_sharded(
            np.asfortranarray(X), y, beta, 0, p, 0.5, tau, sig2, t, 11, 0, lambda v: v, hyper,
            know_tau=True)
        d = np.linalg.norm(got["beta"][t - 1] - beta) / np.linalg.norm(beta)
        assert d < 1e-11, (t, d)


def _alpha_worker(rank, world, port, p, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(9)
    beta = rng.standard_normal(p) * np.exp(rng.uniform(-4, 1, p))
    per = (p + world - 1) // world
    j0, j1 = rank * per, min(p, (rank + 1) * per)

    def allreduce(v):
        t = torch.from_numpy(np.ascontiguousarray(v))
        dist.all_reduce(t)
        return t.numpy()

    out = []
    a = 0.5
    for t in range(1, 40):
        a = gibbs.alpha_mh_sharded(a, beta[j0:j1], p, 0.7, 1.0, 1.0, 13, 2, t, allreduce)
        out.append(a)
    if rank == 0:
        np.save(out_path, np.array(out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_alpha_mh_matches_unsharded(tmp_path, world):
    """The alpha MH step on column shards (its two sums all-reduced, the global p in the
    likelihood) walks the same alpha path as the unsharded oracle step."""
    import oracle

    p = 500
    out = str(tmp_path / "alpha.npy")
    mp.spawn(_alpha_worker, args=(world, _free_port(), p, out), nprocs=world, join=True)
    got = np.load(out)
    rng = np.random.default_rng(9)
    beta = rng.standard_normal(p) * np.exp(rng.uniform(-4, 1, p))
    a, ref = 0.5, []
    for t in range(1, 40):
        a = oracle.alpha_mh(a, beta, 0.7, 1.0, 1.0, 13, 2, t)
        ref.append(a)
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=0)
    assert len(set(np.round(ref, 12))) > 3  # the walk moves
