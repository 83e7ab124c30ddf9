"""Native host code under AddressSanitizer / UndefinedBehaviorSanitizer.

The reference has no sanitizer coverage.  The native wire-frame validator
(``csrc/host/wire_frame.cpp``), which parses bytes received from untrusted
peers, is compiled with ``-fsanitize=address,undefined`` and driven by a
fuzzer (``tests/native/fuzz_wire.cpp``): truncations at every length, payload
bit flips (must be caught by the CRC32C), hostile length fields and garbage.
The HIP kernels' host launchers validate shapes before launch and are covered
by the GPU numerics tests; GPU sanitizers are not available on this pool.
"""

from __future__ import annotations

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("san", ["address,undefined"])
def test_wire_frame_validator_under_sanitizers(tmp_path, san):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = tmp_path / "fuzz_wire"
    cmd = [cxx, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
           os.path.join(ROOT, "csrc", "host", "wire_frame.cpp"), os.path.join(ROOT, "tests", "native", "fuzz_wire.cpp"),
           "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(exe), "1500"], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout


def test_python_and_native_validators_agree():
    """The ctypes-loaded validator and its pure-Python twin accept/reject the same frames."""
    import random
    from collections import OrderedDict

    import torch

    from p2pfl_amd.learning import wire
    from p2pfl_amd.learning.exceptions import DecodingParamsError

    if wire._native() is None:
        pytest.skip("native frame library not built")
    good = wire.encode_params(OrderedDict(w=torch.randn(333), b=torch.arange(7, dtype=torch.int64)))
    rnd = random.Random(0)
    cases = [good, good[:-1], good[:30], b"P2FA" + bytes(40)]
    for _ in range(40):
        g = bytearray(good)
        g[rnd.randrange(len(g))] ^= 1 << rnd.randrange(8)
        cases.append(bytes(g))

    def outcome(data, native):
        saved = wire._lib
        wire._lib = saved if native else False
        try:
            return ("ok", {k: v.tolist() for k, v in wire.decode_params(data).items()})
        except DecodingParamsError as e:
            return ("err", str(e).split(":")[0])
        finally:
            wire._lib = saved

    for c in cases:
        assert outcome(c, True)[0] == outcome(c, False)[0]
