"""Overlap-save tiling geometry (irdu_amd/tiling.py) on CPU: cores partition the image,
windows lie inside it and are aligned, and a pixel-local model is reproduced exactly."""
import pytest
import torch

from irdu_amd import tiling


@pytest.mark.parametrize("hw,tile,halo,align", [((2048, 2048), 256, 32, 16), ((512, 768), 256, 64, 16),
                                                ((96, 200), 64, 16, 2), ((100, 60), 128, 32, 16)])
def test_cores_partition_and_windows_inside(hw, tile, halo, align):
    h, w = hw
    cover = torch.zeros(h, w, dtype=torch.int32)
    for wr, wc, r0, r1, c0, c1 in tiling.tile_grid(h, w, tile, halo, align):
        th, tw = min(tile, h), min(tile, w)
        assert 0 <= wr and wr + th <= h and 0 <= wc and wc + tw <= w
        assert wr <= r0 < r1 <= wr + th and wc <= c0 < c1 <= wc + tw
        assert wr % align == 0 and wc % align == 0
        cover[r0:r1, c0:c1] += 1
    assert bool((cover == 1).all())


def test_pixel_local_model_is_exact():
    img = torch.rand(2, 3, 160, 224)
    model = lambda x: 2.0 * x + 1.0  # noqa: E731
    out = tiling.tiled_forward(model, img, tile=64, halo=16, align=16, micro_batch=5)
    assert torch.equal(out, model(img))


def test_bad_geometry_rejected():
    with pytest.raises(ValueError):
        tiling.tile_grid(512, 512, 256, 128, 16)     # no core left
    with pytest.raises(ValueError):
        tiling.tile_grid(500, 512, 256, 32, 16)      # side not aligned


def _tile_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        conv = torch.nn.Conv2d(3, 2, 3, padding=1, padding_mode="replicate", bias=False)
        torch.nn.init.constant_(conv.weight, 0.1)
        res = {}
        for b in (1, 3):          # one image: windows sharded; three: whole images + a split one
            img = torch.rand(b, 3, 96, 128)
            with torch.no_grad():
                whole = conv(img)
                full = tiling.tiled_forward(conv, img, tile=64, halo=16, align=16, micro_batch=2, out_channels=2,
                                            gather="rank0")
                local = tiling.tiled_forward(conv, img, tile=64, halo=16, align=16, micro_batch=2, out_channels=2)
            wins = tiling.tile_grid(96, 128, 64, 16, 16)
            own = torch.zeros(b, 1, 96, 128)
            for bi, wi in tiling.rank_units(b, len(wins), rank, world):
                _, _, r0, r1, c0, c1 = wins[wi]
                own[bi, :, r0:r1, c0:c1] = 1.0
            res[b] = (None if full is None else float((full - whole).abs().max()),
                      float(((local - whole) * own).abs().max()), float((local * (1 - own)).abs().max()),
                      float(own.sum()))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_window_sharding_over_ranks_without_collective():
    """gloo world 2: each rank filters its share of the (image, window) units and returns its own
    cores with no collective; gather="rank0" assembles the whole image on rank 0 from the packed cores
    alone (a 3x3 replicate-padded conv: receptive field < halo)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tile_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for b in (1, 3):
        assert res[0][b][0] <= 1e-6 and res[1][b][0] is None
        for r in (0, 1):
            assert res[r][b][1] <= 1e-6 and res[r][b][2] == 0.0      # own cores right, nothing else written
        assert res[0][b][3] + res[1][b][3] == b * 96 * 128               # the shares partition the pixels


def test_units_shard_whole_images_first():
    wins = tiling.tile_grid(2048, 2048, 256, 32, 16)
    for world in (2, 4, 8):
        for rank in range(world):
            units = tiling.rank_units(8, len(wins), rank, world)
            assert {bi for bi, _ in units} == set(range(rank * 8 // world, (rank + 1) * 8 // world))
