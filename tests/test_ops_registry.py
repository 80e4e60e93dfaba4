"""CPU checks of the torch-op boundary (specenh/ops.py): every C-ABI compute entry point
is a ``torch.ops.specenh`` operator with a schema and a fake kernel; CPU tensors are
refused (no fallback); shapes propagate through meta tensors without a GPU."""
import pytest
import torch

import specenh  # noqa: F401  (registers the operators)

OPS = ["stft_psd", "stft_psd_out", "csd", "svd_denoise", "svd_denoise_out", "svd_denoise_optimal",
       "conv2d", "conv2d_out", "conv2d_wgrad", "conv2d_wgrad_out", "conv2d_wgrad_pooled_out", "conv2d_pooled_in_out", "convt_conv_out",
       "convt_conv_out_out", "convt_conv_out_train_out", "decoder3", "decoder3_out", "encoder2", "encoder2_out", "maxpool2",
       "maxpool2_out",
       "maxpool2_bwd", "maxpool2_bwd_out", "bce_logits", "bce_logits_out", "adam_step_", "adam_step_flip_",
       "weight_flip_transpose", "weight_flip_transpose_out", "cast", "cast_out", "label_filter",
       "quantfilt", "gaussblr", "morph", "strips_pack", "strips_unpack", "strips_pack_out",
       "strips_unpack_out", "svd_denoise_optimal_out"]

# C-ABI compute entry point -> operator(s) that reach it
CABI = {"specenh_stft_psd": "stft_psd_out", "specenh_stft_psd_f16": "stft_psd_out",
        "specenh_csd": "csd", "specenh_svd_denoise_ex": "svd_denoise_out",
        "specenh_svd_denoise_optimal": "svd_denoise_optimal_out", "specenh_conv2d": "conv2d_out",
        "specenh_conv2d_wgrad": "conv2d_wgrad_out",
        "specenh_conv2d_wgrad_pooled": "conv2d_wgrad_pooled_out",
        "specenh_conv2d_pooled_in": "conv2d_pooled_in_out",
        "specenh_conv2d_wgrad_ex": "conv2d_wgrad_out",
        "specenh_convt_conv_out": "convt_conv_out_out",
        "specenh_convt_conv_out_train": "convt_conv_out_train_out", "specenh_decoder3_ex": "decoder3_out",
        "specenh_encoder2": "encoder2_out",
        "specenh_maxpool2_fwd": "maxpool2_out",
        "specenh_maxpool2_bwd": "maxpool2_bwd_out", "specenh_bce_logits": "bce_logits_out",
        "specenh_adam_step": "adam_step_", "specenh_adam_step_flip": "adam_step_flip_",
        "specenh_weight_flip_transpose":
        "weight_flip_transpose_out", "specenh_cast": "cast_out", "specenh_filter": "label_filter",
        "specenh_quantfilt": "quantfilt", "specenh_gaussblr": "gaussblr",
        "specenh_morph": "morph", "specenh_strips_pack": "strips_pack_out",
        "specenh_strips_unpack": "strips_unpack_out"}


def test_every_operator_is_registered():
    for name in OPS:
        op = getattr(torch.ops.specenh, name)
        assert op.default._schema.name == f"specenh::{name}"


def test_every_compute_entry_point_has_an_operator():
    from test_capi import declared_functions
    host_only = {"specenh_last_error", "specenh_version", "specenh_stft_frames",
                 "specenh_stft_plan_create", "specenh_stft_plan_destroy",
                 "specenh_stft_workspace_bytes", "specenh_csd_plan_create",
                 "specenh_csd_plan_destroy", "specenh_svd_workspace_bytes",
                 "specenh_svd_denoise_workspace_bytes", "specenh_svd_optimal_workspace_bytes",
                 "specenh_conv2d_wgrad_workspace_bytes", "specenh_filter_workspace_bytes",
                 "specenh_u8filter_workspace_bytes", "specenh_set_variant",
                 "specenh_get_variant", "specenh_last_kernel_name", "specenh_launch_count", "specenh_kernel_name_at",
                 "specenh_stream_wait",
                 "specenh_svd_denoise",  # = specenh_svd_denoise_ex with an fp32 output
                 "specenh_decoder3"}  # = specenh_decoder3_ex with an fp32 output
    compute = [n for n in declared_functions() if n not in host_only]
    assert sorted(compute) == sorted(CABI)
    for name in CABI.values():
        assert name in OPS


def test_cpu_tensors_are_refused():
    x = torch.zeros(2, 4096)
    with pytest.raises(NotImplementedError):
        torch.ops.specenh.stft_psd(x, 256, 128, "hann", 500000.0, 0, 2, 1e-11, 7)
    with pytest.raises(NotImplementedError):
        torch.ops.specenh.maxpool2(torch.zeros(1, 4, 4, 2))


def test_meta_shapes():
    m = torch.device("meta")
    S = torch.ops.specenh.stft_psd(torch.empty(3, 16512, device=m), 256, 128, "hann", 5e5, 0, 2,
                                   1e-11, 7)
    assert S.shape == (3, 128, 128) and S.dtype == torch.float32
    y = torch.ops.specenh.conv2d(torch.empty(2, 16, 16, 8, device=m, dtype=torch.bfloat16),
                                 torch.empty(16 * 25 * 8, device=m, dtype=torch.bfloat16), None,
                                 5, 5, 16, 1, 1, 1, 2, 32, 32, 1)
    assert y.shape == (2, 32, 32, 16) and y.dtype == torch.bfloat16
    p, am = torch.ops.specenh.maxpool2(torch.empty(2, 8, 6, 4, device=m))
    assert p.shape == (2, 4, 3, 4) and am.dtype == torch.uint8
    o, ns, med = torch.ops.specenh.svd_denoise_optimal(torch.empty(5, 64, 48, device=m), 0)
    assert o.shape == (5, 64, 48) and ns.dtype == torch.int32 and med.dtype == torch.float64
    st = torch.ops.specenh.strips_pack(torch.empty(2, 256, 3905, device=m), 256, 128, 30,
                                       torch.bfloat16)
    assert st.shape == (60, 256, 128, 1) and st.dtype == torch.bfloat16
