"""Host-compiled checks of boundary helpers shared with the device code
(dragonboat_amd/csrc): each is a small C++ program under tests/host/, built
with g++ and run here."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.parametrize("name", ["upd_has_check"])
def test_host_check(tmp_path, name):
    exe = tmp_path / name
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "dragonboat_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"), "-o", str(exe),
                    os.path.join(HERE, "host", name + ".cpp")], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
