"""Dynamic loss scaling with ``torch.cuda.amp.GradScaler`` semantics, fully on device.

Reference: `distributed_syncBN_amp.py:196,275-278` (``GradScaler(enabled=use_amp)``, ``scale(loss)
.backward()``, ``step``, ``update``) with the upstream defaults (`T/amp/grad_scaler.py:126-129`):
init scale 2**16, growth x2 every 2000 overflow-free steps, backoff x0.5 on overflow, step skipped
on overflow.

Unlike the upstream scaler there is no host synchronisation: the scale lives in a device tensor that
the fused cross-entropy kernel reads (the backward seed is multiplied by it), ``found_inf`` is a
device flag written by a non-finite scan of the flat gradient buffer, the fused SGD kernel reads it
to skip the step, and the growth/backoff update is a one-thread kernel.
"""
from __future__ import annotations

import torch


class DeviceGradScaler:
    def __init__(self, device, enabled: bool = True, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000):
        self.enabled = enabled
        self.device = torch.device(device)
        self.growth_factor = growth_factor
        self.backoff_factor = backoff_factor
        self.growth_interval = growth_interval
        self._scale = torch.full((1,), init_scale if enabled else 1.0, dtype=torch.float32, device=self.device)
        self._tracker = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._found_inf = torch.zeros(1, dtype=torch.float32, device=self.device)

    @property
    def scale_tensor(self):
        return self._scale if self.enabled else None

    @property
    def found_inf(self):
        return self._found_inf if self.enabled else None

    def get_scale(self) -> float:
        return float(self._scale.item()) if self.enabled else 1.0

    def unscale_check(self, grad_flat: torch.Tensor) -> None:
        """Set ``found_inf`` if any (still scaled) gradient is non-finite."""
        if not self.enabled:
            return
        self._found_inf.zero_()
        if grad_flat.is_cuda:
            from ..ops import native
            native.C.nonfinite_check(grad_flat, self._found_inf)
        else:
            if not torch.isfinite(grad_flat).all():
                self._found_inf.fill_(1.0)

    def update(self) -> None:
        if not self.enabled:
            return
        if self._scale.is_cuda:
            from ..ops import native
            native.C.amp_update(self._scale, self._tracker, self._found_inf, self.growth_factor, self.backoff_factor,
                                self.growth_interval)
        else:
            if self._found_inf.item() != 0:
                self._scale.mul_(self.backoff_factor)
                self._tracker.zero_()
            else:
                self._tracker.add_(1)
                if int(self._tracker.item()) == self.growth_interval:
                    self._scale.mul_(self.growth_factor)
                    self._tracker.zero_()

    def state_dict(self) -> dict:
        if not self.enabled:
            return {}
        return {"scale": self.get_scale(), "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval, "_growth_tracker": int(self._tracker.item())}

    def load_state_dict(self, sd: dict) -> None:
        if not sd or not self.enabled:
            return
        self._scale.fill_(float(sd["scale"]))
        self._tracker.fill_(int(sd.get("_growth_tracker", 0)))
        self.growth_factor = sd.get("growth_factor", self.growth_factor)
        self.backoff_factor = sd.get("backoff_factor", self.backoff_factor)
        self.growth_interval = sd.get("growth_interval", self.growth_interval)
