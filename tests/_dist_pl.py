"""Rank script for tests/test_gpu_dist.py: kwhisper.pseudo_label under torch.distributed.run with the RCCL
("nccl") backend -- init_process_group(device_id=...), the per-round width all_reduce(MAX) and id all_gathers
(gather="round", run_pseudo_labelling.py:339-341) and the deferred exchange (gather="end") -- and the ASR
pipeline's data-parallel window batches, over the tiny bf16 engine, against the same calls without a process
group.  Prints one JSON line on rank 0."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    from kwhisper.config import TINY, generation_constants
    from kwhisper.feature_extraction import WhisperFeatureExtractor
    from kwhisper.generation import KWhisperForConditionalGeneration
    from kwhisper.pseudo_label import pseudo_label
    from kwhisper.synthetic import reazon_audio, reazon_durations, synthetic_state_dict

    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    model = KWhisperForConditionalGeneration.from_state_dict(TINY, synthetic_state_dict(TINY, 0), dtype=torch.bfloat16,
                                                             device=dev, generation_config=generation_constants(TINY))
    fe = WhisperFeatureExtractor(feature_size=TINY.num_mel_bins, device=dev)
    n, bs = 10, 4
    durs = reazon_durations()[:n]
    audio = np.zeros((n, 480000), np.float32)
    for i, d in enumerate(durs):
        c = reazon_audio(i, float(d))
        audio[i, : len(c)] = c
    audio = torch.from_numpy(audio).to(dev)

    def features(idx):
        return fe.extract(audio[list(idx)])

    kw = dict(language="ja", task="transcribe", return_timestamps=True, max_length=48)
    pad = model.generation_config.eos_token_id
    ref_ids, ref = pseudo_label(model, features, n, batch_size=bs, gen_kwargs=kw, pad_token_id=pad)  # no group yet
    dist.init_process_group("nccl", device_id=dev)
    out = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    for mode in ("round", "end"):
        ids, preds = pseudo_label(model, features, n, batch_size=bs, gen_kwargs=kw, pad_token_id=pad, gather=mode)
        out[mode] = bool(ids == ref_ids and len(preds) == len(ref) and all(np.array_equal(a, b) for a, b in zip(preds, ref)))
    # the ASR pipeline's window batches under the process group (config 5 at W GPUs): one gather at the end
    from kwhisper.pipeline import ASRPipeline

    clips = [{"array": reazon_audio(50 + i, 40.0 - 9 * i), "sampling_rate": 16000} for i in range(3)]
    kwp = dict(chunk_length_s=15, batch_size=2, generate_kwargs=dict(language="ja", task="transcribe", max_length=32))
    dp = ASRPipeline(model, data_parallel=True, **kwp)(clips, return_timestamps=True)
    single = ASRPipeline(model, data_parallel=False, **kwp)(clips, return_timestamps=True)
    out["pipeline"] = json.dumps(dp, default=str) == json.dumps(single, default=str)
    dist.barrier()
    dist.destroy_process_group()
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
