"""The training engine end to end on the GPU: run_train's YAMLs train through the HIP forward +
reverse kernels, write the reference's checkpoint dict and resume from it.
experiment_conf/example.yaml is config C1 as BASELINE.json states it (single-scale GLR, 1 stage,
64x64 gray, sigma 25, batch 1); experiment_conf/example_v1x0_small.yaml is a small two-scale v1.0
AbtractMultiScaleGraphFilter on the reference YAML's own values (sigma 15, batch 4)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def T():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    from irdu_amd import training
    return training


def test_run_train_example_v1x0_yaml_and_resume(T, tmp_path):
    conf = T.parse_options(os.path.join(ROOT, "experiment_conf", "example_v1x0_small.yaml"))
    conf["path"]["root_dir"] = str(tmp_path)
    conf["train"].update(total_iters=4, checkpoint_every=2, verbose_every=1)
    conf["datasets"]["train"]["dataset_args"]["max_num_patchs"] = 64
    conf["train"]["val_every"] = 2
    tr = T.run(conf, device=torch.device("cuda:0"))
    assert tr.i == 4
    # the reference's periodic test (reflect-pad to x16 of 100 x 140, crop, ubyte PSNR) ran on the HIP model
    assert [i for i, _ in tr.val_history] == [2, 4] and all(np.isfinite(p) for _, p in tr.val_history), tr.val_history
    ck = sorted(os.listdir(T.checkpoint_dir(conf)))
    assert ck == ["checkpoint_iter00000002.pt", "checkpoint_iter00000004.pt"]
    # the graph filters received gradients and moved
    lf = tr.model.localfilter_scale_00.local_filter
    assert lf.alphaCGD.grad is not None and float(lf.alphaCGD.grad.abs().sum()) > 0
    conf["train"]["total_iters"] = 6
    tr2 = T.run(conf, device=torch.device("cuda:0"))
    assert tr2.i == 6
    saved = torch.load(os.path.join(T.checkpoint_dir(conf), "checkpoint_iter00000006.pt"), weights_only=True)
    assert saved["i"] == 6 and set(saved) == {"i", "model", "optimizer", "lr_scheduler"}
    assert all(np.isfinite(v.float().cpu().numpy()).all() for v in saved["model"].values())


def test_c1_example_yaml_trains_and_matches_oracle(T, tmp_path):
    """Config C1 end to end: the example.yaml model (GLRImageFilter, G = 4, F = 1, S = 1) trains
    on 64x64 gray sigma-25 patches at batch 1 through run_train's loop; the trained filter's
    forward on a fresh patch then matches the CPU oracle (1e-4 relative, PSNR within 0.01 dB)."""
    from oracle import graph_oracle as O
    conf = T.parse_options(os.path.join(ROOT, "experiment_conf", "example.yaml"))
    ds_args = conf["datasets"]["train"]["dataset_args"]
    assert (ds_args["patch_size"], ds_args["lambda_noise"], ds_args["n_channels"]) == (64, 25.0, 1)
    assert conf["datasets"]["train"]["dataloader_args"]["batch_size"] == 1
    assert conf["model"]["type"] == "GLRImageFilter" and conf["model"]["args"]["n_cgd_iters"] == 1
    conf["path"]["root_dir"] = str(tmp_path)
    conf["train"].update(total_iters=6, checkpoint_every=3, verbose_every=1)
    tr = T.run(conf, device=torch.device("cuda:0"))
    assert tr.i == 6
    m = tr.model.eval()
    lf = m.localfilter
    assert lf.alphaCGD.grad is not None and float(lf.alphaCGD.grad.abs().sum()) > 0
    ds = T.SyntheticNoisyPatches(lambda_noise=25.0, patch_size=64, max_num_patchs=4, n_channels=1, seed=99)
    noisy, clean = (t.permute(2, 0, 1)[None].contiguous() for t in ds[0])
    p = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref = O.glr_image_filter(noisy, p, m.ngraphs)
    with torch.no_grad():
        got = m(noisy.cuda()).cpu()
    err = float((got.double() - ref.double()).abs().max() / ref.double().abs().max())
    assert err <= 1e-4, err
    assert abs(O.psnr_ubyte(got, clean) - O.psnr_ubyte(ref, clean)) <= 0.01


def test_run_train_multiblocks_v7_yaml(T, tmp_path):
    """The multiblocks script's model (REF7 MultiScaleSequenceDenoiser: 24 graphs x 3 features,
    5x5 diamond, feature CNN 128 wide) trains through run_train on the window-graph HIP reverse:
    finite loss, every solver parameter receives a gradient, the reference's checkpoint dict."""
    conf = T.parse_options(os.path.join(ROOT, "experiment_conf", "multiblocks_v7.yaml"))
    assert conf["model"]["type"] == "MultiScaleSequenceDenoiser"
    conf["path"]["root_dir"] = str(tmp_path)
    conf["train"].update(total_iters=3, checkpoint_every=3, verbose_every=1)
    conf["datasets"]["train"]["dataset_args"].update(max_num_patchs=16, patch_size=32)
    conf["datasets"]["train"]["dataloader_args"]["batch_size"] = 2
    tr = T.run(conf, device=torch.device("cuda:0"))
    assert tr.i == 3
    mix = tr.model.mixtureGLR_block03
    for name in ("alphaCGD", "betaCGD", "ro00", "muys00", "gamma00"):
        g = getattr(mix, name).grad
        assert g is not None and bool(torch.isfinite(g).all()), name
    for mod in (mix.GTVmodule00, mix.GLRmodule00):
        assert mod.multiM.grad is not None and float(mod.multiM.grad.abs().sum()) > 0
        assert mod.stats_kernel_p03.grad is not None
    saved = torch.load(os.path.join(T.checkpoint_dir(conf), "checkpoint_iter00000003.pt"), weights_only=True)
    assert set(saved) == {"i", "model", "optimizer", "lr_scheduler"}
    assert all(np.isfinite(v.float().cpu().numpy()).all() for v in saved["model"].values())
