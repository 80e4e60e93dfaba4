"""Time BASELINE config 3 (4096 x 513 x 256 fp32, rank-16 / default) on the GPU: the
bench's own C3 stage (gapped matrices, SURVEY.md §8 d) as a standalone command."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

print(json.dumps(bench.svd_c3_stage(torch.device("cuda"), B=int(os.environ.get("B", 4096)),
                                     pmc=bench.load_pmc())))
