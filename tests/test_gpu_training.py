"""The training engine end to end on the GPU: run_train's YAML (experiment_conf/example.yaml,
config C1 shapes) trains the v1.0 model through the HIP forward + reverse kernels, writes the
reference's checkpoint dict and resumes from it."""
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


def test_run_train_example_yaml_and_resume(T, tmp_path):
    conf = T.parse_options(os.path.join(ROOT, "experiment_conf", "example.yaml"))
    conf["path"]["root_dir"] = str(tmp_path)
    conf["train"].update(total_iters=4, checkpoint_every=2, verbose_every=1)
    conf["datasets"]["train"]["dataset_args"]["max_num_patchs"] = 64
    tr = T.run(conf, device=torch.device("cuda:0"))
    assert tr.i == 4
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
