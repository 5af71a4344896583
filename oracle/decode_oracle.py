"""CPU oracle for the inference path's greedy CTC decode — TEST INFRASTRUCTURE ONLY.

Restates y00njaekim/CMU-11785-IDL-1.58bit-ASR onebit_asr/metrics.py:51-60
(``ctc_greedy_decode(logits [T, V], blank_id=3)``): argmax per frame (first index on ties,
like torch.argmax), emit a token when it is not blank and differs from the previous frame's
argmax (blank frames update ``prev`` too). Applied per utterance over its valid frames.
"""
from __future__ import annotations

from typing import List

import numpy as np


def np_ctc_greedy_decode(logits: np.ndarray, blank_id: int = 3) -> List[int]:
    pred = np.argmax(np.asarray(logits), axis=-1).tolist()  # metrics.py:53
    out: List[int] = []
    prev = None
    for t in pred:  # metrics.py:55-59
        if t != blank_id and t != prev:
            out.append(int(t))
        prev = t
    return out


def np_ctc_greedy_decode_batch(logits: np.ndarray, lens, blank_id: int = 3) -> List[List[int]]:
    return [np_ctc_greedy_decode(logits[b, :int(n)], blank_id) for b, n in enumerate(lens)]
