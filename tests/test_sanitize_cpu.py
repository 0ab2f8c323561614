"""Host sanitizer pass: the library's CPU code
that parses untrusted bytes -- stream framing (csrc/framing.cpp:
tpf_block_size / tpf_scan_offsets) and the host streams' caller-offset check
(tpf_check_offsets) -- and the oracle's decoders (oracle/tpf_oracle.c) built
with -fsanitize=address,undefined and fed valid, corrupted, truncated and
random streams of five formats by tests/cpp/sanitize_framing.cpp.  Any
out-of-bounds access, leak or undefined behaviour aborts the driver
(-fno-sanitize-recover)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no host compiler")
def test_framing_and_oracle_under_asan_ubsan(tmp_path):
    flags = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]
    orc = tmp_path / "orc.o"
    exe = tmp_path / "san"
    subprocess.check_call(["gcc", *flags, "-std=c11", "-c", os.path.join(ROOT, "oracle", "tpf_oracle.c"), "-o", str(orc)])
    subprocess.check_call(["g++", *flags, "-std=c++20", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "sanitize_framing.cpp"),
                           os.path.join(ROOT, "turbopfor-cpp_amd", "csrc", "framing.cpp"), str(orc), "-o", str(exe)])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), "60"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout
