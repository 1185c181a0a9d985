"""Host sanitizers: the C++ TF-bundle codec built with AddressSanitizer + UndefinedBehaviorSanitizer
and driven by ``csrc/tfbundle/selftest.cpp`` over the reference's own demo checkpoint (CRC vectors, byte-identical
rebuild, every single-byte flip and truncation of the index, 20k random mutations, block handles / tensor extents
whose offset + size overflows). The first run of this test found an out-of-bounds read in ``read_block`` (a
wrapping ``off + size`` bound check), fixed in ``tf_bundle.cpp``. Host code only: GPU sanitizers are not used."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TFB = os.path.join(ROOT, "csrc", "tfbundle")


def test_tfbundle_codec_under_asan_ubsan(tmp_path):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "tfb_selftest")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-static-libasan", "-I", TFB, os.path.join(TFB, "selftest.cpp"),
           os.path.join(TFB, "tf_bundle.cpp"), "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, os.path.join(ROOT, "tests", "fixtures", "model-Pendulum_a3c"), str(tmp_path)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "all checks passed" in r.stdout
