"""Lab scan (``-m "gpu and slow"``, not part of the round's GPU suite): which clips take a SECOND timestamp seek
pass in transformers' fp32 large-v3 at ``max_length`` 128?  The fp32 engine is bit-exact with
transformers on the oracle log-mel (tests/test_gpu_workloads.py), so its per-row pass counts on those features are
transformers'.  Scans the config-4 stand-in clips at their ReazonSpeech-tiny durations and two 30 s kinds; writes
gpurun_out/multipass_scan.json (tools/make_fixtures.py --only large_c4_mp builds the fixture from it).
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

from kwhisper.config import LARGE_V3, generation_constants  # noqa: E402
from kwhisper.synthetic import dummy_audio, reazon_audio, reazon_durations, synthetic_state_dict  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_scan_multipass_clips():
    from kwhisper.generation import KWhisperForConditionalGeneration
    from oracle.mel import log_mel, pad_or_trim

    n = int(os.environ.get("KW_SCAN_CLIPS", "1768"))
    model = KWhisperForConditionalGeneration.from_state_dict(LARGE_V3, synthetic_state_dict(LARGE_V3, 0),
                                                             dtype=torch.float32,
                                                             generation_config=generation_constants(LARGE_V3))
    durs = reazon_durations()
    kinds = {"reazon": [(i, lambda i=i: reazon_audio(i, float(durs[i]))) for i in range(n)],
             "reazon30": [(i, lambda i=i: reazon_audio(i, 30.0)) for i in range(64)],
             "dummy30": [(i, lambda i=i: dummy_audio(i)) for i in range(64)]}
    out = {}
    for kind, items in kinds.items():
        passes = []
        for b0 in range(0, len(items), 32):
            chunk = items[b0: b0 + 32]
            feats = torch.from_numpy(log_mel(np.stack([pad_or_trim(f()) for _, f in chunk]), 128)).cuda()
            model.generate(feats, language="ja", task="transcribe", return_timestamps=True, max_length=128)
            passes += model.stats["row_passes"].tolist()
            print(f"{kind} {b0}: multi-pass so far {[i for i, p in enumerate(passes) if p >= 2]}", flush=True)
        out[kind] = {"passes": passes, "multipass": [i for i, p in enumerate(passes) if p >= 2]}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "multipass_scan.json"), "w") as f:
        json.dump(out, f)
    print({k: v["multipass"] for k, v in out.items()})
