"""The C++ adapter (orc_amd/csrc/GpuRleDecoder.hh) compiled as a reference-
style host program: compiles on CPU; runs the KATs through it on the GPU."""
import os
import subprocess

import pytest

from conftest import ROOT, load_golden

SRC = os.path.join(ROOT, "tests", "cxx", "adapter_test.cpp")
OUT = os.path.join(ROOT, "tests", "cxx", "build", "adapter_test")


def build_adapter_test():
    from orc_amd import build as orc_build

    orc_build.build()
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.check_call([
        "g++", "-std=c++17", "-O2", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", SRC, "-o", OUT,
        "-L" + os.path.join(ROOT, "orc_amd"), "-lorcgpu", "-Wl,-rpath," + os.path.join(ROOT, "orc_amd"),
        "-Wl,-rpath,/opt/rocm/lib",
    ])
    return OUT


def test_adapter_compiles_and_links():
    assert os.access(build_adapter_test(), os.X_OK)


def _fixture_lines():
    lines = []
    for fx in load_golden("kat_rlev2.json"):
        if "not_null" in fx:
            continue
        exp = ["x" if e is None else str(e) for e in fx["expected"]]
        lines.append("rlev2 %d %s %d %s" % (int(fx["signed"]), fx["data"], len(exp), " ".join(exp)))
    for name, kind in (("kat_byterle.json", "byte"), ("kat_boolrle.json", "bool")):
        for fx in load_golden(name):
            if "not_null" in fx:
                continue
            exp = ["x" if e is None else str(e) for e in fx["expected"]]
            lines.append("%s 0 %s %d %s" % (kind, fx["data"], len(exp), " ".join(exp)))
    return lines


@pytest.mark.gpu
def test_adapter_kats_on_gpu(tmp_path):
    exe = build_adapter_test()
    f = tmp_path / "kats.txt"
    f.write_text("\n".join(_fixture_lines()) + "\n")
    r = subprocess.run([exe, str(f)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("OK")
