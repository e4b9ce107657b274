"""Measurement tool (not product): device sin / cos / acos (tools/libm_probe.hip, the device
math library) and the device form of the glibc restatement (ompl_amd/csrc/glibc_sincos.h)
against the host's glibc on the hot path's argument ranges.

    python tools/libm_probe.py [n]   (runs tools/libm_probe, writes gpurun_out/libm_probe.json)"""
import ctypes
import json
import math
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


_libm = ctypes.CDLL("libm.so.6")
_libm.sincos.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
_libm.sincos.restype = None


def _sincos(v):
    s, c = ctypes.c_double(), ctypes.c_double()
    _libm.sincos(v, ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    rng = np.random.default_rng(1)
    sets = {"chain_theta_12pi": rng.uniform(-12 * math.pi, 12 * math.pi, n),
            "unit_interval": rng.uniform(0.0, 1.0, n),
            "near_one": 1.0 - np.ldexp(rng.uniform(0.0, 1.0, n), -rng.integers(5, 50, n))}
    out = {}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for name, x in sets.items():
        fi, fo = f"/tmp/libm_in_{name}.bin", f"/tmp/libm_out_{name}.bin"
        x.astype(np.float64).tofile(fi)
        subprocess.run([os.path.join(HERE, "libm_probe"), fi, fo], check=True)
        y = np.fromfile(fo, dtype=np.float64).reshape(8, n)
        res = {}
        sc = np.array([_sincos(v) for v in x])  # glibc's sincos
        for k, fn in enumerate(("sin", "cos", "acos", "glibc_sin", "glibc_cos", "glibc_sincos_s", "glibc_sincos_c",
                            "glibc_acos")):
            if fn.endswith("acos") != (name != "chain_theta_12pi"):
                continue
            if fn.startswith("glibc_sincos"):
                ref = sc[:, 0 if fn.endswith("_s") else 1]
            else:
                f = getattr(math, fn.replace("glibc_", ""))
                if fn.endswith("acos"):
                    f = lambda v: math.acos(v if abs(v) <= 1.0 else 0.5)  # noqa: E731
                ref = np.array([f(v) for v in x])  # glibc
            diff = y[k] != ref
            ulps = np.abs(y[k] - ref) / np.spacing(np.abs(ref))
            res[fn] = {"n": n, "mismatch": int(diff.sum()), "rate": float(diff.mean()), "max_ulps": float(ulps.max())}
        out[name] = res
    print(json.dumps(out, indent=1))
    with open(os.path.join(ROOT, "gpurun_out", "libm_probe.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
