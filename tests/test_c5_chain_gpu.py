"""BASELINE config 5 as a chain on the GPU vs the fp64 CPU chain (SURVEY.md §8 d, C5).

fp16 shots (16,512 samples) -> specgr straight from fp16 (256 hann / hop 128, linear,
density, log, min-max, drop Nyquist) -> denoiseSignal default stored as fp16 -> fp16
autoencoder forward with the trained reference-model weights, exactly the bench's stream,
compared shot by shot with scipy-semantics specgr (oracle, fp64) -> numpy-SVD
denoiseSignal -> fp64 autoencoder restatement on the same fp16 samples.

Tolerance: out_rel (error over the output's own spread) <= checks.TOL['float16'] per
shot; the intermediate spectrograms within the fp32 STFT contract (1e-5 max abs)."""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import autoencoder as ora
from oracle import checks
from oracle import svd as osvd
from oracle.spectrogram import specgr_arrays

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))

SPEC5 = {"nperseg": 256, "noverlap": 128, "fs": 500000, "window": "hann",
         "scaling": "density", "detrend": "linear", "eps": 1e-11}
L5 = 16512


def _engine(dev, ws):
    from specenh import ae
    C, P = ae.ConvOp, ae.PoolOp
    ops = [C("conv", 1, 16, 5, "relu"), P(), C("conv", 16, 32, 5, "relu"), P(),
           C("conv", 32, 64, 5, "relu"), P(), C("convT", 64, 64, 5, "relu", stride=2),
           C("convT", 64, 32, 5, "relu", stride=2), C("convT", 32, 16, 5, "relu", stride=2),
           C("conv", 16, 1, 5, "sigmoid")]
    eng = ae.AutoencoderEngine(ops, (128, 128, 1), compute_dtype="float16", device=dev)
    eng.set_keras_weights(ws)
    return eng


@pytest.mark.parametrize("streams", [1, 2])
def test_c5_chain_matches_cpu_chain(gpu_device, streams):
    from make_ae_weights import load
    from specenh import pipeline_data, svd
    from specenh.synthetic import plasma_chirps

    ws = load()
    B = 8
    x16 = plasma_chirps(B, L5, seed0=4242, dtype=np.float16)
    xd = torch.as_tensor(x16, device=gpu_device)
    S = torch.empty((B, 128, 128), dtype=torch.float32, device=gpu_device)
    A = torch.empty((B, 128, 128, 1), dtype=torch.float16, device=gpu_device)
    engs = [_engine(gpu_device, ws) for _ in range(streams)]
    outs = []
    h = B // streams
    sts = [torch.cuda.Stream(gpu_device) for _ in range(streams)]
    for i in range(streams):  # the bench's per-stream slices
        sts[i].wait_stream(torch.cuda.current_stream(gpu_device))
        with torch.cuda.stream(sts[i]):
            sl = slice(i * h, (i + 1) * h)
            pipeline_data.specgr_batch(xd[sl], SPEC5, out=S[sl])
            svd.denoise_batch(S[sl], out=A[sl].view(h, 128, 128))
            outs.append(engs[i].forward(A[sl]).clone())
    torch.cuda.synchronize()
    Y = torch.cat(outs).double().cpu().numpy()
    Sg = S.double().cpu().numpy()
    spec = ora.ae_spec()
    it, params = iter(ws), []
    for lay in spec:
        params.append(None if lay[0] == "pool" else
                      {"W": torch.tensor(next(it), dtype=torch.float64),
                       "b": torch.tensor(next(it), dtype=torch.float64)})
    errs = []
    for b in range(B):
        Sx, _, _ = specgr_arrays(x16[b].astype(np.float64), SPEC5)
        assert np.abs(Sg[b] - Sx).max() <= 1e-5
        D = osvd.denoiseSignal(Sx)
        with torch.no_grad():
            ref = ora.forward(spec, params, torch.from_numpy(D)[None, :, :, None]).numpy()[0]
        errs.append(checks.out_rel(Y[b], ref))
        assert np.std(ref) > 0.1  # the trained model's output carries a signal
    print("C5 chain out_rel per shot:", ["%.1e" % e for e in errs])
    assert max(errs) <= checks.TOL["float16"]["out_rel"], errs


def test_c5_chain_at_bench_launch_shape(gpu_device):
    """The bench's own 2048-shot launch (bench.make_c5_engine: fused decoder, persistent and
    wave-split variants, the one-pass SVD), every buffer poisoned with NaN first, checked
    against the fp64 CPU chain on shots spread over the launch: both ends, the middle, and
    positions that fall in different workgroups of each persistent grid."""
    import bench
    from specenh import pipeline_data, svd
    from specenh.synthetic import plasma_chirps_torch

    B = 2048
    x = plasma_chirps_torch(B, L5, seed=777, device=gpu_device, dtype=torch.float16)
    S = torch.full((B, 128, 128), float("nan"), dtype=torch.float32, device=gpu_device)
    A = torch.full((B, 128, 128, 1), float("nan"), dtype=torch.float16, device=gpu_device)
    eng = bench.make_c5_engine(gpu_device)
    for lst in eng._buffers(B, False).values():  # every activation buffer of this launch
        for t in (lst if isinstance(lst, list) else [lst]):
            if torch.is_tensor(t) and t.is_floating_point():
                t.fill_(float("nan"))
    pipeline_data.specgr_batch(x, SPEC5, out=S)
    svd.denoise_batch(S, out=A.view(B, 128, 128))
    Y = eng.forward(A).float()
    torch.cuda.synchronize()
    assert torch.isfinite(Y).all()
    shots = [0, 1, 511, 512, 1023, 1024, 1337, 2046, 2047]
    xs = x[shots].double().cpu().numpy()
    Yg = Y[shots].double().cpu().numpy()
    Sg = S[shots].double().cpu().numpy()
    ws = bench.ae_weights()
    spec = ora.ae_spec()
    it, params = iter(ws), []
    for lay in spec:
        params.append(None if lay[0] == "pool" else
                      {"W": torch.tensor(next(it), dtype=torch.float64),
                       "b": torch.tensor(next(it), dtype=torch.float64)})
    errs = []
    for j in range(len(shots)):
        Sx, _, _ = specgr_arrays(xs[j], SPEC5)
        assert np.abs(Sg[j] - Sx).max() <= 1e-5
        D = osvd.denoiseSignal(Sx)
        with torch.no_grad():
            ref = ora.forward(spec, params, torch.from_numpy(D)[None, :, :, None]).numpy()[0]
        errs.append(checks.out_rel(Yg[j], ref))
    print("C5 launch-shape out_rel:", ["%.1e" % e for e in errs])
    assert max(errs) <= checks.TOL["float16"]["out_rel"], errs
