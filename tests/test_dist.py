"""CPU multi-process test of the N>1 path (gloo, world_size 2 and 3): each
rank computes its slice's partial MSM (C oracle stands in for the GPU), the
partials are all-gathered and folded by halo2-aggregation_amd/sharded.py with
the library's host pm_points_sum (one call per fold, sharded.points_fold)
exactly as in bench.py, and every rank must hold the full MSM."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_per_rank, q, host_collectives=False):
    import sys

    for p in (ROOT, os.path.join(ROOT, "halo2-aggregation_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import halo2_amd as H
    import msm_ref
    import pasta as P
    from sharded import PartialPipe, combine_partials, points_fold, shard_range

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if host_collectives:  # bench.py's PM_BENCH_SHARE_GPU rehearsal wrapper
        import bench

        dist = bench.HostCollectives(dist, torch)
        t = torch.tensor([rank + 1.0])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        assert t.item() == world
    i0, n = shard_range(rank, world, n_per_rank)
    S = msm_ref.synth_scalars(0, P.SEED_SCALARS, i0, n, threads=2)
    B = msm_ref.synth_bases(0, P.SEED_BASES, i0, n, threads=2)
    part = msm_ref.best_multiexp(0, S, B, threads=2)

    padd = points_fold(0)  # the fold bench.py runs: one pm_points_sum call

    full = combine_partials(part, dist, torch.device("cpu"), padd, world)
    # bench.py's pipelined form (sharded.PartialPipe): step k returns step
    # k - 1's fold, drain() the last one -- every step must equal the full MSM
    pipe = PartialPipe(dist, torch.device("cpu"), padd, world)
    piped = [pipe.step(part) for _ in range(3)] + [pipe.drain()]
    assert piped[0] is None and pipe.drain() is None
    q.put((rank, [int(x) for x in full], [[int(x) for x in r] for r in piped[1:]]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,host_collectives", [(2, False), (3, False), (2, True)])
def test_sharded_msm_gloo(world, host_collectives):
    import msm_ref
    import pasta as P

    n_per_rank = 700
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_per_rank, q, host_collectives))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    res = {r: full for r, full, _ in got}
    piped = {r: p for r, _, p in got}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = world * n_per_rank
    S = msm_ref.synth_scalars(0, P.SEED_SCALARS, 0, n, threads=4)
    B = msm_ref.synth_bases(0, P.SEED_BASES, 0, n, threads=4)
    want = [int(x) for x in msm_ref.best_multiexp(0, S, B, threads=4)]
    for r in range(world):
        assert res[r] == want, r
        assert piped[r] == [want] * 3, r


def test_split_range_covers():
    from sharded import split_range

    for n in (0, 1, 7, 1000, 1 << 20):
        for w in (1, 2, 3, 8):
            parts = [split_range(r, w, n) for r in range(w)]
            assert sum(c for _, c in parts) == n
            assert all(parts[i][0] + parts[i][1] == parts[i + 1][0] for i in range(w - 1) if parts[i + 1][1])


def _accum_worker(rank, world, port, B, q):
    import sys

    for p in (os.path.join(ROOT, "halo2-aggregation_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import accum as A
    import accum_util as U
    import transcript as T
    from sharded import gather_batches

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    C, sh, proofs = U.make_case(2, "simple", 10, world * B, 0xD15)
    mine = proofs[rank * B:(rank + 1) * B]           # rank r owns proofs [rB, (r+1)B)
    T.with_replayed_challenges(C, sh, mine, T.vk_repr(C.r, b"vk"))
    quads = np.stack([A.pack_result(C, A.accumulate_msm(C, sh, pf))[0] for pf in mine])
    full = gather_batches(torch.from_numpy(quads.view(np.int64)), dist, world)
    q.put((rank, full.numpy().view(np.uint64).tolist()))
    dist.destroy_process_group()


def test_sharded_accumulator_gloo():
    """Proof-batch sharding of the accumulator (bench.py's accumulator leg):
    every rank ends with all world x B quads, in rank order, equal to the
    oracle on the whole batch."""
    import sys

    for p in (os.path.join(ROOT, "halo2-aggregation_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import accum as A
    import accum_util as U
    import transcript as T

    world, B = 2, 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_accum_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    C, sh, proofs = U.make_case(2, "simple", 10, world * B, 0xD15)
    T.with_replayed_challenges(C, sh, proofs, T.vk_repr(C.r, b"vk"))
    want = np.stack([A.pack_result(C, A.accumulate_msm(C, sh, pf))[0] for pf in proofs])
    for r in range(world):
        assert np.array_equal(np.array(res[r], dtype=np.uint64), want), r


def test_bench_launcher_world2():
    """bench.py --gpus 2 without a torch.distributed environment starts 2
    ranks through torch.distributed.run (child process), the ranks check
    WORLD_SIZE == --gpus, rendezvous over gloo (--dry-run: no GPU work) and
    rank 0 prints ONE JSON line with n_gpus == 2."""
    import json
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3"],
                       capture_output=True, text=True, timeout=240, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3


def test_bench_world_mismatch_refused():
    """A rank whose WORLD_SIZE differs from --gpus refuses to report."""
    import subprocess
    import sys

    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd="/tmp")
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_accum_multi_shard_math_cpu():
    """pm_accum_batch_multi's split (context k takes [k*ceil(B/n), ...), the
    same ranges as sharded.split_range) on a ragged batch: running the C
    accumulator port (oracle/accum_ref.c) per range and concatenating equals
    the whole batch, challenges, quads, h_eval and status included."""
    import sys

    for p in (os.path.join(ROOT, "halo2-aggregation_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import accum as A
    import accum_ref as R
    import accum_util as U
    from sharded import split_range

    C, sh, proofs = U.make_case(2, "simple", 10, 7, 0xA77)
    ps = U.to_product_shape(2, sh)
    pts, scs, _ = A.pack_proofs(C, sh, proofs)
    vk = np.array(A.to_limbs_mont(C.r, 99), dtype=np.uint64)
    whole = R.accum_batch(2, ps.c, pts, scs, vk_repr=vk, threads=2)
    for nctx in (1, 2, 3, 4, 8):
        parts = [split_range(k, nctx, 7) for k in range(nctx)]
        got = [[], [], [], []]
        for lo, cnt in parts:
            if cnt == 0:
                continue
            out = R.accum_batch(2, ps.c, pts[lo:lo + cnt], scs[lo:lo + cnt], vk_repr=vk, threads=1)
            for i in range(4):
                got[i].append(out[i])
        for i in range(4):
            assert np.array_equal(np.concatenate(got[i]), whole[i]), (nctx, i)


@pytest.mark.parametrize("curve", [0, 1, 2])
def test_points_sum_one_call(curve):
    """pm_points_sum (the partials' fold) equals the oracle's sum and the
    pairwise pm_point_add fold, including the identity, a repeated point
    (doubling), P + (-P) and n = 0 / 1."""
    import sys

    for p in (os.path.join(ROOT, "halo2-aggregation_amd"), os.path.join(ROOT, "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import halo2_amd as H
    import pasta as P

    C = (P.PALLAS, P.VESTA, P.BN254)[curve]
    pts = [C.mul(7 + 3 * i, C.gen) for i in range(6)]
    neg = C.neg(pts[2]) if hasattr(C, "neg") else C.mul(C.r - 9 - 6, C.gen)
    cases = [[], [pts[0]], pts, pts + [None, pts[1]], [pts[3], pts[3]], [pts[2], neg], [None, None]]
    for case in cases:
        rows = np.array([P.point_to_limbs(C, q) for q in case], dtype=np.uint64).reshape(-1, 8)
        got = H.points_sum(curve, rows)
        acc = np.zeros(8, dtype=np.uint64)
        want = None
        for r, q in zip(rows, case):
            acc = H.point_add(curve, acc, r)
            want = q if want is None else (C.add(want, q) if q is not None else want)
        assert np.array_equal(got, acc), case
        assert P.limbs_to_point(C, [int(v) for v in got]) == want, case
