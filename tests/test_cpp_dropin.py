"""Compile a C++ program against include/nova_crc32c.hpp and link libnova_crc32c.so,
as NovaLSM would; run the util/crc32c_test.cc cases."""
import os
import subprocess

from novalsm_amd import crc32c as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_dropin(tmp_path):
    C.load(build_if_missing=True)
    lib_dir = os.path.dirname(C.lib_path())
    exe = str(tmp_path / "dropin_test")
    subprocess.run(["g++", "-std=c++11", "-O2", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "dropin_test.cc"), "-o", exe,
                    "-L", lib_dir, "-lnova_crc32c", f"-Wl,-rpath,{lib_dir}"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "PASSED" in r.stdout
