"""Warm-up learning-rate wrappers with the reference's semantics
(DRT/trainer/scheduler.py:24-133): step() sets the lr for step n (1-based)
then steps the wrapped optimizer; linear warm-up from init_lr to max_lr over
n_warmup_steps, then inverse-sqrt / cosine / linear / constant."""
from __future__ import annotations

import math


class AbstractScheduler:
    def __init__(self, base_optimizer, init_lr: float):
        self.optimizer = base_optimizer
        self.init_lr = init_lr
        self.n_steps = 0

    def step(self):
        self.n_steps += 1
        lr = self.lr
        for g in self.optimizer.param_groups:
            g["lr"] = lr
        self.optimizer.step()

    @property
    def lr(self):
        raise NotImplementedError

    def state_dict(self):
        return self.optimizer.state_dict(), self.n_steps

    def load_state_dict(self, state):
        opt, self.n_steps = state
        self.optimizer.load_state_dict(opt)

    def __getattr__(self, item):
        return getattr(self.optimizer, item)


class _Warmup(AbstractScheduler):
    def __init__(self, base_optimizer, init_lr, max_lr, n_warmup_steps, max_steps=None):
        super().__init__(base_optimizer, init_lr)
        self.max_lr = max_lr
        self.n_warmup_steps = n_warmup_steps
        self.max_steps = max_steps
        self.warmup_k = (max_lr - init_lr) / n_warmup_steps

    def _warm(self):
        return self.init_lr + self.warmup_k * self.n_steps


class InverseSquareRootScheduler(_Warmup):
    @property
    def lr(self):
        if self.n_steps <= self.n_warmup_steps:
            return self._warm()
        return self.max_lr * math.sqrt(self.n_warmup_steps) / math.sqrt(self.n_steps)


class CosineScheduler(_Warmup):
    @property
    def lr(self):
        if self.n_steps <= self.n_warmup_steps:
            return self._warm()
        t = (self.n_steps - self.n_warmup_steps) * math.pi / (self.max_steps - self.n_warmup_steps)
        return self.init_lr + (self.max_lr - self.init_lr) / 2 * (1.0 + math.cos(t))


class LinearScheduler(_Warmup):
    @property
    def lr(self):
        if self.n_steps <= self.n_warmup_steps:
            return self._warm()
        k = (self.max_lr - self.init_lr) / (self.max_steps - self.n_warmup_steps)
        return self.max_lr - k * (self.n_steps - self.n_warmup_steps)


class ConstantScheduler(_Warmup):
    @property
    def lr(self):
        if self.n_steps <= self.n_warmup_steps:
            return self._warm()
        return self.max_lr
