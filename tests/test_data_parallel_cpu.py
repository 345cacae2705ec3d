"""parallel.data_parallel.DataParallel: the single-device entry main.py / main_dist.py wrap the net in
(reference main.py:73-74 ``net = torch.nn.DataParallel(net)``). Several GPUs are one rank per GPU
(parallel.launcher + parallel.ddp), covered by test_cli_cpu / test_ddp_cpu."""
import pytest
import torch


def test_checkpoint_layout_and_forward():
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.parallel.data_parallel import DataParallel

    torch.manual_seed(0)
    m = models.LeNet()
    dp = DataParallel(m)
    assert dp.device_ids == []   # CPU model: no device ids
    sd = dp.state_dict()
    assert list(sd) == ["module." + k for k in m.state_dict()]   # nn.DataParallel's `module.` keys
    x = torch.randn(2, 3, 32, 32)
    assert torch.equal(dp(x), m(x))
    # a reference-layout checkpoint (module.-prefixed) loads strictly into the wrapper
    m2 = models.LeNet()
    dp2 = DataParallel(m2)
    dp2.load_state_dict(sd, strict=True)
    assert torch.equal(dp2(x), m(x))


def test_several_devices_in_one_process_rejected():
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.parallel.data_parallel import DataParallel

    with pytest.raises(ValueError, match="one rank per GPU"):
        DataParallel(models.LeNet(), device_ids=[0, 1])
    assert DataParallel(models.LeNet(), device_ids=[0]).device_ids == [0]
