"""The GPU's sin/cos restatement (csrc/heist_trig.h) vs the host libm, bit for bit.

CPU: the header compiled with g++ against ~10^7 inputs across every branch
(tests/native/trig_check.cpp).  GPU: heist_sincos vs math.sin / math.cos on ray angles
and random arguments."""
import math
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "rl-project-heist-architect-adversarial-reinforcement-learning-framework-cse4019_amd", "csrc")


def test_host_restatement_bit_exact(tmp_path):
    exe = str(tmp_path / "trig_check")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-I", CSRC,
                    os.path.join(HERE, "native", "trig_check.cpp"), "-o", exe, "-lm"], check=True)
    r = subprocess.run([exe, "2000000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "bad 0" in r.stdout


def _inputs():
    rng = np.random.default_rng(0)
    d2r = np.pi / 180.0
    xs = [rng.uniform(-10, 10, 400000), np.arange(-200000, 800000) * 0.001 * d2r]
    fov = rng.uniform(30, 120, 2000).astype(np.float32).astype(np.float64)
    head = rng.uniform(0, 360, 2000)
    k = np.arange(0, 241)
    nr = np.maximum((fov * 2).astype(np.int64), 30)
    ang = ((head - fov / 2.0)[:, None] + (fov[:, None] * k[None, :]) / nr[:, None])
    xs.append((ang[k[None, :] <= nr[:, None]]) * d2r)
    return np.concatenate(xs)


@pytest.mark.gpu
def test_device_sincos_bit_exact(gpu_device):
    import torch
    from heist_amd import _native as nat
    x = _inputs()
    xt = torch.from_numpy(x).to(gpu_device)
    so = torch.empty_like(xt)
    co = torch.empty_like(xt)
    nat.check(nat.lib().heist_sincos(nat.ptr(xt), xt.numel(), nat.ptr(so), nat.ptr(co), nat.stream(gpu_device)),
              "heist_sincos")
    # math.sin/math.cos (host libm, exactly what the reference calls); numpy may use SIMD kernels
    s_ref = np.array([math.sin(v) for v in x.tolist()])
    c_ref = np.array([math.cos(v) for v in x.tolist()])
    assert np.array_equal(so.cpu().numpy().view(np.int64), s_ref.view(np.int64))
    assert np.array_equal(co.cpu().numpy().view(np.int64), c_ref.view(np.int64))
