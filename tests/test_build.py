"""The in-tree extension must link (no undefined symbols) and expose the full kernel API."""


def test_extension_imports_and_exports():
    from pytorch_cifar_amd import _native

    C = _native.lib()
    for name in ["conv_fwd", "conv_dgrad", "conv_wgrad", "weight_prep", "bn_stats", "bn_finalize",
                 "bn_apply", "bn_backward", "augment", "gap_fwd", "gap_bwd", "avgpool_fwd",
                 "maxpool_fwd", "ce_fused", "sgd_step", "se_scale_fwd", "dw_fwd", "dw_dgrad",
                 "dw_wgrad", "direct_fwd", "direct_dgrad", "direct_wgrad", "RcclComm",
                 "rccl_unique_id", "set_conv_tile"]:
        assert hasattr(C, name), name
