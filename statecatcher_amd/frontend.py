"""The reference's feature frontend, ``make_frontend`` (model.py:250-279), on the GPU.

``make_frontend("mfcc" | "mel", sample_rate)`` returns ``(module, mel_kwargs)`` like the
reference.  The module maps audio ``[..., time]`` to features ``[..., 80, frames]`` exactly as
torchaudio's ``MFCC(n_mfcc=80, dct_type=2, norm="ortho", log_mels=True, melkwargs)`` or
``Sequential(MelSpectrogram(**melkwargs), AmplitudeToDB(top_db=80))`` do, so train.py's
``frontend(batch).transpose(1, 2)`` (train.py:473-475) is unchanged; the computation is one
HIP kernel (csrc/fbank.hip, ``sc_fbank``) that writes the transposed ``[B, frames, 80]``
layout directly (the module returns it as a transposed view).

AmplitudeToDB packs dim -3 when the spectrogram has more than two dims, so its top_db floor is
relative to the max over the last three dims: over the whole batch for ``[B, time]`` audio, per
leading item for ``[B, C, time]`` — both reproduced here.
"""
import torch
import torch.nn as nn

from .ops import fbank

MEL_KWARGS = {"n_fft": 400, "win_length": 400, "hop_length": 160, "n_mels": 80, "center": False,
              "power": 2.0, "mel_scale": "htk"}


class GPUFrontend(nn.Module):
    def __init__(self, kind: str, sample_rate: int):
        super().__init__()
        if kind not in ("mfcc", "mel"):
            raise ValueError(f"Unsupported frontend: {kind}")
        self.kind, self.sample_rate = kind, sample_rate

    def forward(self, audio: torch.Tensor) -> torch.Tensor:
        lead = audio.shape[:-1]
        if self.kind == "mel" and audio.dim() > 2:
            # top_db per item of dims [:-2]: one call per item (each covers a [C, time] block)
            x = audio.reshape(-1, audio.shape[-2], audio.shape[-1])
            out = torch.stack([fbank(x[i], self.kind, self.sample_rate) for i in range(x.shape[0])])
        else:
            out = fbank(audio.reshape(-1, audio.shape[-1]), self.kind, self.sample_rate)
        return out.reshape(*lead, out.shape[-2], 80).transpose(-1, -2)


def make_frontend(ftype: str, sample_rate: int):
    """model.py:250-279: (frontend module, mel kwargs)."""
    if ftype not in ("mfcc", "mel"):
        raise ValueError(f"Unsupported frontend: {ftype}")
    return GPUFrontend(ftype, sample_rate), dict(MEL_KWARGS)
