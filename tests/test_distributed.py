"""Multi-rank frame path on CPU (gloo), world sizes 2 and 3.

Every rank renders only its round-robin row stripes (stripes.rank_rows) into a
slab, the slabs are gathered to rank 0 with ONE collective (frame.gather_slabs,
the same call bench.py makes over RCCL), and rank 0 restores row order
(stripes.unshuffle, the numpy twin of the rt_unshuffle_stripes kernel).  The
per-stripe renderer here is the CPU oracle (row-range render), so the test runs
without a GPU; the assembled frame must be bit-identical to the reference
golden.  The device twin of this test is test_gpu_parity.py::test_stripes_*.
"""
from __future__ import annotations

import hashlib
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN_DIR, ROOT, golden_by_name


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, xml, stripe_rows, aa, out_json):
    import sys

    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as graft

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = graft.import_pkg()
        orc = graft.import_oracle()
        sc = orc.OracleScene(xml)
        W, H, _ = sc.cameras()[0]
        rows = pkg.stripes.rank_rows(H, stripe_rows, world, rank)
        slab = np.zeros((len(rows), W, 3), dtype=np.uint8)
        # this rank's stripes only: contiguous runs of global rows
        lr = 0
        while lr < len(rows):
            g0 = rows[lr]
            if g0 < 0:
                break
            n = 1
            while lr + n < len(rows) and rows[lr + n] == g0 + n:
                n += 1
            img, _ = sc.render(0, aa=aa, threads=2, rows=(int(g0), int(g0) + n))
            slab[lr:lr + n] = img
            lr += n
        sc.close()
        frame = pkg.frame.assemble_frame(torch.from_numpy(slab), H, stripe_rows)
        # a 3-frame batch (bench --inflight): frames slab, 255 - slab, slab in one gather
        batch = torch.from_numpy(np.stack([slab, 255 - slab, slab]))
        frames = pkg.frame.assemble_frames(batch, H, stripe_rows)
        if rank == 0:
            arr = frame.numpy()
            sha = lambda a: hashlib.sha256(a.tobytes()).hexdigest()  # noqa: E731
            with open(out_json, "w") as f:
                json.dump({"shape": list(arr.shape), "sha256": sha(arr),
                           "batch": [sha(frames[0].numpy()), sha(255 - frames[1].numpy()), sha(frames[2].numpy())]},
                          f)
        else:
            assert frame is None and frames is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,stripe_rows", [(2, 8), (3, 24)])
def test_gloo_stripes_gather_bit_exact(world, stripe_rows, goldens, scene_dir, tmp_path):
    g = golden_by_name(goldens, "C1_simple_aa1")
    cam = g["cameras"][0]
    out = tmp_path / "frame.json"
    xml = str(scene_dir / "C1_simple.xml")
    mp.start_processes(_rank_main, args=(world, _free_port(), xml, stripe_rows, 1, str(out)), nprocs=world,
                       join=True, start_method="spawn")
    res = json.loads(out.read_text())
    assert res["shape"] == [cam["height"], cam["width"], 3]
    assert res["sha256"] == cam["sha256_rgb"]
    assert res["batch"] == [cam["sha256_rgb"]] * 3


def test_gather_single_rank_is_identity(pkg):
    slab = torch.arange(2 * 5 * 3, dtype=torch.uint8).reshape(2, 5, 3)
    g = pkg.frame.gather_slabs(slab)
    assert g.shape == (1, 2, 5, 3) and torch.equal(g[0], slab)
    img = pkg.frame.assemble_frame(slab, 2, 8)
    assert torch.equal(img, slab)


@pytest.mark.parametrize("H,S,N", [(1080, 8, 8), (1080, 8, 3), (7, 8, 2), (800, 24, 3), (1, 1, 4)])
def test_stripe_partition_covers_every_row_once(pkg, H, S, N):
    seen = np.concatenate([pkg.stripes.rank_rows(H, S, N, r) for r in range(N)])
    seen = seen[seen >= 0]
    assert np.array_equal(np.sort(seen), np.arange(H))
    assert pkg.stripes.slab_rows(H, S, N) * N >= H
    # the slab layout and the unshuffle are inverse permutations
    W = 2
    img = np.random.default_rng(H + S + N).integers(0, 256, (H, W, 3), dtype=np.uint8)
    slabs = np.zeros((N, pkg.stripes.slab_rows(H, S, N), W, 3), dtype=np.uint8)
    for r in range(N):
        rows = pkg.stripes.rank_rows(H, S, N, r)
        ok = rows >= 0
        slabs[r][ok] = img[rows[ok]]
    assert np.array_equal(pkg.stripes.unshuffle(slabs, H, S), img)


def _cams_main(rank, world, port, xml, out_json):
    import sys

    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as graft

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = graft.import_pkg()
        orc = graft.import_oracle()
        sc = orc.OracleScene(xml)
        cams = sc.cameras()
        sizes = [(h, w) for (w, h, _) in cams]
        own = pkg.frame.camera_ranks(len(cams), world)
        local = {}
        for i in range(len(cams)):
            if own[i] == rank:                       # this rank's cameras only
                img, _ = sc.render(i, aa=1, threads=2)
                local[i] = torch.from_numpy(img)
        sc.close()
        imgs = pkg.frame.gather_camera_images(local, sizes, device="cpu")
        if rank == 0:
            with open(out_json, "w") as f:
                json.dump([hashlib.sha256(im.numpy().tobytes()).hexdigest() for im in imgs], f)
        else:
            assert imgs is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_camera_batch_gather(world, goldens, scene_dir, tmp_path):
    # (f4) cameras dealt round-robin over ranks (4 ranks > 3 cameras: one rank idle), one gather
    g = golden_by_name(goldens, "cornellbox_aa1")
    out = tmp_path / "cams.json"
    xml = str(scene_dir / "cornellbox.xml")
    mp.start_processes(_cams_main, args=(world, _free_port(), xml, str(out)), nprocs=world, join=True,
                       start_method="spawn")
    shas = json.loads(out.read_text())
    assert shas == [c["sha256_rgb"] for c in g["cameras"]]


def test_camera_ranks_round_robin(pkg):
    assert pkg.frame.camera_ranks(5, 2) == [0, 1, 0, 1, 0]
    assert pkg.frame.camera_ranks(3, 8) == [0, 1, 2]
