"""Learning-rate schedules + optimizer selection, drop-in for estimator/define_optimizer.py.

The update itself is the fused HIP kernel (``seg_apply_update``); this module resolves the
per-step learning rate exactly as tf.train.piecewise_constant / polynomial_decay do, the
momentum (MomentumOptimizer, optionally Nesterov) or 0 (GradientDescentOptimizer).
"""
from dataclasses import dataclass
from typing import List


@dataclass
class Optimizer:
    schedule: str
    boundaries: List[int]
    values: List[float]
    initial: float
    final: float
    power: float
    decay_steps: int
    momentum: float
    use_nesterov: bool

    def learning_rate(self, global_step: int) -> float:
        if self.schedule == 'piecewise_constant':
            # tf.train.piecewise_constant: values[i] for boundaries[i-1] < step <= boundaries[i]
            for b, v in zip(self.boundaries, self.values):
                if global_step <= b:
                    return float(v)
            return float(self.values[len(self.boundaries)])
        # tf.train.polynomial_decay (cycle=False)
        step = min(global_step, self.decay_steps)
        frac = 1.0 - step / float(self.decay_steps)
        return float((self.initial - self.final) * frac ** self.power + self.final)

    # reference code reads optimizer._learning_rate for summaries
    @property
    def _learning_rate(self):
        return self.learning_rate


def define_optimizer(global_step, params):
    if params.learning_rate_schedule not in ('piecewise_constant', 'polynomial_decay'):
        print('Unknown option for learning rate schedule.')
    if params.optimizer == 'SGDM':
        momentum = params.momentum
    elif params.optimizer == 'SGD':
        momentum = 0.0
    else:
        assert False, 'Unknown option for optimizer.'
    return Optimizer(schedule=params.learning_rate_schedule,
                     boundaries=list(getattr(params, 'learning_rate_boundaries', []) or []),
                     values=list(getattr(params, 'learning_rate_values', []) or []),
                     initial=params.learning_rate_initial,
                     final=params.learning_rate_final, power=params.learning_rate_power,
                     decay_steps=max(int(getattr(params, 'num_training_steps', 1)), 1),
                     momentum=momentum,
                     use_nesterov=params.optimizer == 'SGDM' and bool(getattr(params, 'use_nesterov', False)))


class DynamicLossScaler:
    """fp16 loss scaling (BASELINE config C5: fp16 storage with fp32 master gradients), the
    usual dynamic policy: start at 2**16; a step whose loss-scaled gradients overflow is
    skipped on the device (seg_apply_update) and halves the scale; `growth_interval` clean
    steps double it. `update(ctx)` reads the device overflow flag of the step just issued."""

    def __init__(self, ctx, init_scale=2.0 ** 16, growth_interval=2000, backoff=0.5, growth=2.0,
                 min_scale=1.0):
        self.ctx, self.scale, self.growth_interval = ctx, float(init_scale), growth_interval
        self.backoff, self.growth, self.min_scale = backoff, growth, min_scale
        self.good_steps, self.skipped, self.last_overflow = 0, 0, False
        ctx.set_loss_scale(self.scale)

    def update(self):
        flag = self.ctx.found_inf()
        overflow = bool(int(flag.item())) if flag is not None else False
        self.last_overflow = overflow
        if overflow:
            self.skipped += 1
            self.good_steps = 0
            self.scale = max(self.scale * self.backoff, self.min_scale)
        else:
            self.good_steps += 1
            if self.good_steps % self.growth_interval == 0:
                self.scale *= self.growth
        self.ctx.set_loss_scale(self.scale)
        return overflow
