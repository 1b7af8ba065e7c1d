"""Value schedules over timesteps (reference: rllib/utils/schedules/*): exploration epsilons,
learning-rate / entropy-coefficient decays. ``schedule(t)`` == ``schedule.value(t)``."""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple


class Schedule:
    def __init__(self, framework: Optional[str] = None):
        self.framework = framework

    def value(self, t) -> float:
        raise NotImplementedError

    def __call__(self, t) -> float:
        return self.value(t)


class ConstantSchedule(Schedule):
    def __init__(self, value: float, framework: Optional[str] = None):
        super().__init__(framework)
        self._v = float(value)

    def value(self, t):
        return self._v


class PolynomialSchedule(Schedule):
    """``final + (initial - final) * (1 - min(t, T) / T) ** power``."""

    def __init__(self, schedule_timesteps: int, final_p: float, framework: Optional[str] = None,
                 initial_p: float = 1.0, power: float = 2.0):
        super().__init__(framework)
        if schedule_timesteps <= 0:
            raise ValueError("schedule_timesteps must be > 0")
        self.schedule_timesteps = int(schedule_timesteps)
        self.final_p, self.initial_p, self.power = float(final_p), float(initial_p), float(power)

    def value(self, t):
        frac = min(float(t), self.schedule_timesteps) / self.schedule_timesteps
        return self.final_p + (self.initial_p - self.final_p) * (1.0 - frac) ** self.power


class LinearSchedule(PolynomialSchedule):
    def __init__(self, schedule_timesteps: int, final_p: float, framework: Optional[str] = None,
                 initial_p: float = 1.0):
        super().__init__(schedule_timesteps, final_p, framework, initial_p, power=1.0)


class ExponentialSchedule(Schedule):
    """``initial * decay_rate ** (t / T)``."""

    def __init__(self, schedule_timesteps: int, framework: Optional[str] = None, initial_p: float = 1.0,
                 decay_rate: float = 0.1):
        super().__init__(framework)
        if schedule_timesteps <= 0:
            raise ValueError("schedule_timesteps must be > 0")
        self.schedule_timesteps, self.initial_p, self.decay_rate = int(schedule_timesteps), initial_p, decay_rate

    def value(self, t):
        return float(self.initial_p * self.decay_rate ** (float(t) / self.schedule_timesteps))


def _linear_interpolation(l, r, alpha):
    return l + alpha * (r - l)


class PiecewiseSchedule(Schedule):
    """Interpolates between ``endpoints`` [(t, value), ...] (increasing t); outside them
    ``outside_value`` (default: the nearest endpoint's value)."""

    def __init__(self, endpoints: Sequence[Tuple[int, float]], framework: Optional[str] = None,
                 interpolation=_linear_interpolation, outside_value: Optional[float] = None):
        super().__init__(framework)
        ts = [e[0] for e in endpoints]
        if ts != sorted(ts):
            raise ValueError("PiecewiseSchedule endpoints must be sorted by time")
        self.endpoints: List[Tuple[int, float]] = [(int(t), float(v)) for t, v in endpoints]
        self.interpolation = interpolation
        self.outside_value = outside_value

    def value(self, t):
        for (l_t, l), (r_t, r) in zip(self.endpoints[:-1], self.endpoints[1:]):
            if l_t <= t < r_t:
                return float(self.interpolation(l, r, float(t - l_t) / (r_t - l_t)))
        if self.outside_value is not None:
            return float(self.outside_value)
        return self.endpoints[0][1] if t < self.endpoints[0][0] else self.endpoints[-1][1]


class Scheduler:
    """``lr`` / ``entropy_coeff`` given as a constant or as ``[[t0, v0], [t1, v1], ...]``
    (reference rllib/utils/schedules/scheduler.py)."""

    def __init__(self, fixed_value_or_schedule, framework: Optional[str] = "torch"):
        if isinstance(fixed_value_or_schedule, (list, tuple)):
            self._s = PiecewiseSchedule(fixed_value_or_schedule, framework,
                                        outside_value=fixed_value_or_schedule[-1][-1])
        else:
            self._s = ConstantSchedule(fixed_value_or_schedule, framework)
        self._t = 0

    @staticmethod
    def validate(fixed_value_or_schedule, setting_name: str = "", description: str = ""):
        if isinstance(fixed_value_or_schedule, (list, tuple)):
            if not fixed_value_or_schedule or fixed_value_or_schedule[0][0] != 0:
                raise ValueError(f"{setting_name} schedule must start at timestep 0")

    def get_current_value(self) -> float:
        return self._s.value(self._t)

    def update(self, timestep: int) -> float:
        self._t = int(timestep)
        return self.get_current_value()


__all__ = ["Schedule", "ConstantSchedule", "PolynomialSchedule", "LinearSchedule", "ExponentialSchedule",
           "PiecewiseSchedule", "Scheduler"]
