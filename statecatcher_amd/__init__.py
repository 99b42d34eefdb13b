"""statecatcher_amd — MI355X-native hot path of the statecatcher stateful recurrent ASR step.

LucyRNN gated scan (fwd + bwd), decay scan, CTC alpha-beta (+ fused log_softmax) and greedy
CTC decode as hand-written HIP kernels for gfx950 behind a C ABI (include/statecatcher.h),
wrapped in drop-ins of the reference's module API (lucyrnn_triton.py, decoder.py, model.py).
"""
from .lucyrnn_conf import LucyRNNConfig
from .lucyrnn_triton import LinearSafe, LucyRNNCellTriton, LucyRNNtriton
from .lucyrnn import LucyRNN, LucyRNNCell
from .xlstm import xLSTMLarge, xLSTMLargeConfig
from .model import (ASRModel, CTCLoss, RNNTCompactPredictorJoiner, RNNTLoss, RNNTPredictorJoiner,
                    build_lucyrnn_config, build_xlstm_config, compute_loss, detach_states)
from .ops import (ctc_greedy_decode, ctc_loss, ctc_nll, decay_scan, lucy_scan, mlstm_chunkwise,
                  rnnt_loss)
from .decoder import ctc_greedy_decoder
from .streaming import StreamingLucyRNN
from .frontend import make_frontend

__all__ = [
    "LucyRNNConfig", "LinearSafe", "LucyRNNCellTriton", "LucyRNNtriton", "LucyRNN", "LucyRNNCell", "ASRModel", "CTCLoss",
    "compute_loss", "detach_states", "build_lucyrnn_config", "build_xlstm_config", "ctc_greedy_decode", "ctc_loss", "ctc_nll", "decay_scan",
    "lucy_scan", "ctc_greedy_decoder", "rnnt_loss", "RNNTLoss", "RNNTPredictorJoiner",
    "RNNTCompactPredictorJoiner", "xLSTMLarge", "xLSTMLargeConfig", "mlstm_chunkwise",
    "StreamingLucyRNN", "make_frontend",
]
