"""Learning-rate schedulers (reference ``python/hetu/lr_scheduler.py:2-142``).

The user calls ``step()`` (once per iteration / epoch, as in the reference);
optimizers read ``get()`` each update, so a scheduler object can be passed as
``learning_rate``.
"""
from __future__ import annotations


class FixedScheduler(object):
    def __init__(self, learning_rate):
        self.learning_rate = learning_rate

    def step(self, *args):
        return self.learning_rate

    def get(self):
        return self.learning_rate

    def state_dict(self):
        return dict(self.__dict__)

    def load_state_dict(self, st):
        self.__dict__.update(st)


class StepScheduler(FixedScheduler):
    """lr *= gamma every ``step_size`` steps, floored at ``ending``."""

    def __init__(self, learning_rate, step_size, gamma=0.1, ending=1e-8):
        assert step_size > 0 and gamma > 0 and ending >= 0 and learning_rate > ending
        super().__init__(learning_rate)
        self.step_size, self.gamma, self.ending = step_size, gamma, ending
        self.cur_step = 0
        self.reach_end = False

    def step(self):
        if self.reach_end:
            return self.ending
        if self.cur_step and self.cur_step % self.step_size == 0:
            self.learning_rate = max(self.learning_rate * self.gamma, self.ending)
            self.reach_end = self.learning_rate <= self.ending
        self.cur_step += 1
        return self.learning_rate


class MultiStepScheduler(FixedScheduler):
    def __init__(self, learning_rate, milestones, gamma=0.1):
        assert list(milestones) == sorted(milestones) and milestones[0] > 0
        super().__init__(learning_rate)
        self.milestones = list(milestones)
        self.gamma = gamma
        self.cur_step = 0

    def step(self):
        if self.milestones and self.cur_step == self.milestones[0]:
            self.milestones.pop(0)
            self.learning_rate *= self.gamma
        self.cur_step += 1
        return self.learning_rate


class ExponentialScheduler(FixedScheduler):
    """Returns the current lr, then decays it by ``gamma`` (floored)."""

    def __init__(self, learning_rate, gamma=0.9, ending=1e-8):
        assert gamma > 0 and ending >= 0 and learning_rate > ending
        super().__init__(learning_rate)
        self.gamma, self.ending = gamma, ending
        self.reach_end = False

    def step(self):
        prev = self.learning_rate
        if not self.reach_end:
            self.learning_rate = max(self.learning_rate * self.gamma, self.ending)
            self.reach_end = self.learning_rate <= self.ending
        return prev


class ReduceOnPlateauScheduler(FixedScheduler):
    """Scale lr by ``factor`` after more than ``patience`` consecutive steps in
    which the metric got worse by more than ``threshold``."""

    def __init__(self, learning_rate, mode='min', factor=0.1, patience=10, threshold=1e-4,
                 threshold_mode='rel', cooldown=0, ending=1e-8):
        assert mode in ('min', 'max') and threshold_mode in ('rel', 'abs')
        assert factor > 0 and patience >= 0 and threshold >= 0 and cooldown >= 0
        assert ending >= 0 and learning_rate > ending
        super().__init__(learning_rate)
        self.mode, self.factor, self.patience = mode, factor, patience
        self.threshold, self.threshold_mode = threshold, threshold_mode
        self.cooldown, self.ending = cooldown, ending
        self.cooldown_left = 0
        self.bad = 0
        self.best = None
        self.reach_end = False

    def _worse(self, value):
        b = self.best
        if self.mode == 'min':
            lim = b * (1 + self.threshold) if self.threshold_mode == 'rel' else b + self.threshold
            return value > lim
        lim = b * (1 - self.threshold) if self.threshold_mode == 'rel' else b - self.threshold
        return value < lim

    def step(self, value):
        if self.reach_end:
            return self.learning_rate
        if self.best is None:
            self.best = value
            return self.learning_rate
        if self.cooldown_left > 0:
            self.cooldown_left -= 1
        elif self._worse(value):
            if self.bad >= self.patience:
                self.bad = 0
                self.learning_rate = max(self.learning_rate * self.factor, self.ending)
                self.reach_end = self.learning_rate <= self.ending
                self.cooldown_left = self.cooldown
            else:
                self.bad += 1
        else:
            self.bad = 0
        self.best = min(self.best, value) if self.mode == 'min' else max(self.best, value)
        return self.learning_rate
