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
        img = torch.rand(1, 3, 96, 128)
        conv = torch.nn.Conv2d(3, 2, 3, padding=1, padding_mode="replicate", bias=False)
        torch.nn.init.constant_(conv.weight, 0.1)
        with torch.no_grad():
            out = tiling.tiled_forward(conv, img, tile=64, halo=16, align=16, micro_batch=2, out_channels=2)
            whole = conv(img)
        q.put((rank, float((out - whole).abs().max())))
    finally:
        dist.destroy_process_group()


def test_window_sharding_over_ranks_gathers_whole_image():
    """gloo world 2: each rank filters its share of the windows, the all-reduce of the disjoint
    canvases rebuilds the whole image (a 3x3 replicate-padded conv: receptive field < halo)."""
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
    assert res[0] <= 1e-6 and res[1] <= 1e-6
