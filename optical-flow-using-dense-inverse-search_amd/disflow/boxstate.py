"""Read-only GPU clock and socket-power sampling for the bench line.

A VALU-bound kernel's time follows the shader clock, and on MI355X the clock
follows the 1.4 kW socket power cap, so one box's number is
not comparable with another's without the clock it ran at. This samples the
amdgpu hwmon files of the process's GPU -- ``freq1_input`` (sclk, Hz) and
``power1_input`` (socket power, microwatts) -- from a background thread while a
phase of the bench runs. Nothing is written anywhere; if the files are absent
(no amdgpu sysfs, another driver) every summary is None.
"""
from __future__ import annotations

import glob
import os
import threading
import time


def hwmon_dir(pci_domain: int, pci_bus: int, pci_device: int) -> str | None:
    """The hwmon directory of the amdgpu device at domain:bus:device.0."""
    want = f"{pci_domain:04x}:{pci_bus:02x}:{pci_device:02x}.0"
    for dev in glob.glob("/sys/class/drm/card*/device"):
        try:
            if os.path.basename(os.path.realpath(dev)) != want:
                continue
        except OSError:
            continue
        for h in sorted(glob.glob(os.path.join(dev, "hwmon", "hwmon*"))):
            if os.path.exists(os.path.join(h, "freq1_input")):
                return h
    return None


def torch_hwmon_dir(device_index: int) -> str | None:
    try:
        import torch
        p = torch.cuda.get_device_properties(device_index)
        return hwmon_dir(int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
    except Exception:
        return None


class Sampler:
    """Background sampling of sclk and socket power; ``with s.phase(name):``
    marks a phase, ``summary()`` gives per-phase mean / min / max."""

    def __init__(self, hwmon: str | None, period_s: float = 0.002):
        self.dir = hwmon
        self.period = period_s
        self._fds = {}
        if hwmon:
            for k, f in (("sclk", "freq1_input"), ("power", "power1_input")):
                try:
                    self._fds[k] = os.open(os.path.join(hwmon, f), os.O_RDONLY)
                except OSError:
                    pass
        self._phase = None
        self._samples = {}
        self._stop = threading.Event()
        self._th = None
        if "sclk" in self._fds:
            self._th = threading.Thread(target=self._run, daemon=True)
            self._th.start()

    def _read(self, k):
        try:
            return int(os.pread(self._fds[k], 64, 0).split()[0])
        except (OSError, ValueError, IndexError, KeyError):
            return None

    def _run(self):
        while not self._stop.is_set():
            ph = self._phase
            if ph is not None:
                self._samples.setdefault(ph, []).append((self._read("sclk"), self._read("power")))
            time.sleep(self.period)

    class _Phase:
        def __init__(self, s, name):
            self.s, self.name = s, name

        def __enter__(self):
            self.s._phase = self.name

        def __exit__(self, *exc):
            self.s._phase = None

    def phase(self, name: str):
        return Sampler._Phase(self, name)

    def close(self):
        self._stop.set()
        if self._th:
            self._th.join(timeout=1.0)
        for fd in self._fds.values():
            os.close(fd)
        self._fds = {}

    def summary(self, name: str):
        xs = self._samples.get(name)
        if not xs:
            return None
        cl = [a / 1e6 for a, _ in xs if a]
        pw = [b / 1e6 for _, b in xs if b]
        out = {"samples": len(xs)}
        if cl:
            out.update(sclk_MHz_mean=sum(cl) / len(cl), sclk_MHz_min=min(cl), sclk_MHz_max=max(cl))
        if pw:
            out.update(power_W_mean=sum(pw) / len(pw), power_W_max=max(pw))
        return out
