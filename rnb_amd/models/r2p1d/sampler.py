"""Clip sampler for R(2+1)D (reference: models/r2p1d/sampler.py:1-62).

Given a video length, picks ``num_clips`` (weighted choice from
``num_clips_population``; reference default 1 clip w.p. 10/11, 15 clips w.p.
1/11, so E[clips] = 25/11) and returns the start frame of each clip: clips are
spread over the whole video with equal spacing ``floor(len / n)`` and a random
offset in ``[0, leniency]``; if ``clip_length * n`` exceeds the length the
count is reduced until it fits. Same semantics as the reference, without the
NVVL base class (the loader backends consume the start indices directly).
"""
from __future__ import annotations

import random
from typing import List, Optional, Sequence


class R2P1DSampler:
    def __init__(self, clip_length: int = 8, num_clips: int = 10,
                 num_clips_population: Optional[Sequence[int]] = (1, 15),
                 num_clips_weights: Optional[Sequence[float]] = (10, 1),
                 seed: Optional[int] = None):
        self.clip_length = clip_length
        self.num_clips = num_clips
        self.num_clips_population = list(num_clips_population) if num_clips_population else None
        self.num_clips_weights = list(num_clips_weights) if num_clips_weights else None
        self.rng = random.Random(seed)

    def _sample(self, length: int, num_clips: int) -> Optional[List[int]]:
        while num_clips > 0 and self.clip_length * num_clips > length:
            num_clips -= 1
        if num_clips == 0:
            return None
        stride = int(float(length) / num_clips)
        interval = stride - self.clip_length
        leniency = interval + (length - stride * num_clips)
        start = self.rng.randint(0, leniency)
        return [start + i * stride for i in range(num_clips)]

    def choose_num_clips(self) -> int:
        if self.num_clips_population is not None and self.num_clips_weights is not None:
            return self.rng.choices(self.num_clips_population, self.num_clips_weights)[0]
        return self.num_clips

    def sample(self, length: int) -> Optional[List[int]]:
        return self._sample(length, self.choose_num_clips())

    def expected_clips(self) -> float:
        if self.num_clips_population is None or self.num_clips_weights is None:
            return float(self.num_clips)
        tot = float(sum(self.num_clips_weights))
        return sum(p * w for p, w in zip(self.num_clips_population,
                                         self.num_clips_weights)) / tot
