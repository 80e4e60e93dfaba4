"""The STFT team schedule (csrc/stft_psd.hip stft_team_kernel: a shot's frame tiles on a
team of co-resident workgroups exchanging their extremes through agent-scope granules,
every output byte written once) against the one-workgroup-per-shot kernel with its
normalisation sweep: bitwise identical outputs (same arithmetic, same min/max)."""
import numpy as np
import pytest

from oracle import spectrogram as ref

pytestmark = pytest.mark.gpu
DEV_NOTEAM = 1 << 17
DEV_FORCETEAM = 1 << 18


def _both(x, nperseg, noverlap, window):
    import torch

    from specenh import _lib, stft

    plan = stft.get_plan(x.device, nperseg, noverlap, window, 500000.0, "density", "linear", 1e-11)
    T = stft.frame_count(x.shape[1], nperseg, noverlap)
    flags = _lib.STFT_LOG | _lib.STFT_NORMALIZE | _lib.STFT_DROP_NYQUIST
    outs = []
    for extra in (DEV_FORCETEAM, DEV_NOTEAM):
        out = torch.full((x.shape[0], nperseg // 2, T), float("nan"), device=x.device)
        stft._launch(plan, x, out, flags | extra)
        outs.append(out)
        if extra == DEV_FORCETEAM:  # the team schedule never timed out waiting for a member
            torch.cuda.synchronize()
            assert int(plan.workspace(x.shape[0], x.device)[:4].view(torch.int32)[0]) == 0
    torch.cuda.synchronize()
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
    team, sweep = _both(x, nperseg, noverlap, window)
    assert not team.isnan().any()
    assert (team == sweep).all()
    p = {"nperseg": nperseg, "noverlap": noverlap, "fs": 500000, "window": window,
         "scaling": "density", "detrend": "linear", "eps": 1e-11}
    for b in (0, B - 1):
        truth, _, _ = ref.specgr_arrays(x[b].double().cpu().numpy(), p)
        assert np.abs(team[b].double().cpu().numpy() - truth).max() <= 1e-5
