"""The STFT team schedule (csrc/stft_psd.hip stft_team_kernel: a shot's frame tiles on a
team of co-resident workgroups exchanging their extremes through agent-scope granules,
every output byte written once) against the one-workgroup-per-shot kernel with its
normalisation sweep: bitwise identical outputs (same arithmetic, same min/max). A team
whose wait gives up stores raw tiles that team_fixup_kernel normalises afterwards: also
bitwise identical, so correctness never rests on co-residency."""
import numpy as np
import pytest

from oracle import spectrogram as ref

pytestmark = pytest.mark.gpu
DEV_NOTEAM = 1 << 17
DEV_FORCETEAM = 1 << 18
DEV_GIVEUP = 1 << 19


def _both(x, nperseg, noverlap, window):
    import torch

    from specenh import _lib, stft

    plan = stft.get_plan(x.device, nperseg, noverlap, window, 500000.0, "density", "linear", 1e-11)
    T = stft.frame_count(x.shape[1], nperseg, noverlap)
    flags = _lib.STFT_LOG | _lib.STFT_NORMALIZE | _lib.STFT_DROP_NYQUIST
    outs = []
    for extra in (DEV_FORCETEAM, DEV_NOTEAM, DEV_FORCETEAM | DEV_GIVEUP):
        out = torch.full((x.shape[0], nperseg // 2, T), float("nan"), device=x.device)
        ws = plan.workspace(x.shape[0], x.device)
        # the sweep kernel proper (short shots would otherwise take its held-tile
        # instantiation, whose FFT code is scheduled differently: equal to ~1e-5 only,
        # tests/test_stft_gpu.py::test_held_tiles_match_sweep)
        with _lib.variant("STFT_NO_HOLD", 1):  # restores the caller's value
            stft._launch(plan, x, out, flags | extra, workspace=ws)
        outs.append(out)
        torch.cuda.synchronize()
        tmo = int(ws[:4].view(torch.int32)[0])
        if extra == DEV_FORCETEAM:  # the team schedule never timed out waiting for a member
            assert tmo == 0
        elif extra & DEV_GIVEUP:    # every wait gave up: every tile stored raw, then fixed up
            assert tmo == 1
    return outs


@pytest.mark.parametrize("nperseg,noverlap,window,L,B", [
    (256, 128, "hann", 16512, 4096),      # C5 / C1 parameters: teams of 2
    (1024, 768, "hamm", 65536, 512),      # C2 parameters: teams of 8
    (512, 256, "hamm", 200_000, 64),      # reference parameters, long shots: teams of 13
    (64, 48, "hann", 640, 300),           # one-member teams
    (128, 64, "hamm", 128 * 70 + 17, 33)])  # odd batch vs team slots
def test_team_equals_sweep_kernel(nperseg, noverlap, window, L, B, gpu_device):
    from specenh.synthetic import plasma_chirps_torch

    x = plasma_chirps_torch(B, L, seed=nperseg + B, device=gpu_device)
    team, sweep, fixed = _both(x, nperseg, noverlap, window)
    assert not team.isnan().any()
    assert (team == sweep).all()
    assert (fixed == sweep).all()
    p = {"nperseg": nperseg, "noverlap": noverlap, "fs": 500000, "window": window,
         "scaling": "density", "detrend": "linear", "eps": 1e-11}
    for b in (0, B - 1):
        truth, _, _ = ref.specgr_arrays(x[b].double().cpu().numpy(), p)
        assert np.abs(team[b].double().cpu().numpy() - truth).max() <= 1e-5


def test_team_with_concurrent_conv_stream(gpu_device):
    """The C2 team path on one stream while autoencoder convolutions fill the device from a
    second stream (co-residency can break): output equals the sweep kernel and the fp64
    oracle; any wait that gave up was finished by the fixup pass."""
    import torch

    from specenh import _lib, ae, pipeline_data
    from specenh.synthetic import plasma_chirps_torch

    B, L = 1024, 65536
    p = {"nperseg": 1024, "noverlap": 768, "fs": 500000, "window": "hamm",
         "scaling": "density", "detrend": "linear", "eps": 1e-11}
    x = plasma_chirps_torch(B, L, seed=77, device=gpu_device)
    C, P = ae.ConvOp, ae.PoolOp
    ops = [C("conv", 1, 16, 5, "relu"), P(), C("conv", 16, 32, 5, "relu"), P(),
           C("convT", 32, 16, 5, "relu", stride=2), C("convT", 16, 16, 5, "relu", stride=2),
           C("conv", 16, 1, 5, "sigmoid")]
    eng = ae.AutoencoderEngine(ops, (128, 128, 1), compute_dtype="float16", device=gpu_device)
    xa = torch.rand((2048, 128, 128, 1), device=gpu_device).half()
    s_conv, s_stft = torch.cuda.Stream(gpu_device), torch.cuda.Stream(gpu_device)
    torch.cuda.synchronize()
    outs = []
    for _ in range(3):
        with torch.cuda.stream(s_conv):
            for _ in range(4):
                eng.forward(xa)
        with torch.cuda.stream(s_stft):
            outs.append(pipeline_data.specgr_batch(x, p))
    torch.cuda.synchronize()
    from specenh import stft
    plan = stft.get_plan(x.device, 1024, 768, "hamm", 500000.0, "density", "linear", 1e-11)
    sweep = torch.empty_like(outs[0])
    stft._launch(plan, x, sweep, _lib.STFT_LOG | _lib.STFT_NORMALIZE | _lib.STFT_DROP_NYQUIST
                 | DEV_NOTEAM)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, sweep)
    for b in (0, B - 1):
        truth, _, _ = ref.specgr_arrays(x[b].double().cpu().numpy(), p)
        assert np.abs(outs[0][b].double().cpu().numpy() - truth).max() <= 1e-5
