"""the multi-GPU host streams (tpf_host_dec_multi /
tpf_host_enc_multi) had only ever met one physical device.  Their device
discipline -- each shard thread bound to its device before it runs, every
shard thread joined whatever the others did, pooled pipelines made, handed out
and destroyed only on their own device -- lives in the HIP-free header
turbopfor-cpp_amd/csrc/shard_exec.h, which host_stream.cpp instantiates with
hipSetDevice / hipGetDevice.  This test drives the same header with a mock
device map (tests/cpp/shard_exec_mock.cpp): eight devices, permuted and
repeated device lists, a failing shard, a throwing shard, a device whose
selection fails, and a release from a thread on another device.  Host only,
also under ThreadSanitizer."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "shard_exec_mock.cpp")
INC = os.path.join(ROOT, "turbopfor-cpp_amd", "csrc")


@pytest.mark.parametrize("san", [None, "thread"])
def test_shard_exec_device_discipline(tmp_path, san):
    exe = tmp_path / ("shard_exec" + (("_" + san) if san else ""))
    cmd = ["g++", "-std=c++20", "-O1", "-g", "-Wall", "-Werror", "-I", INC, SRC, "-lpthread", "-o", str(exe)]
    if san:
        cmd.insert(1, "-fsanitize=" + san)
    subprocess.check_call(cmd)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "shard exec ok" in r.stdout
