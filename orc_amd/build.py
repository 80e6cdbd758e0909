"""Build liborcgpu.so in-tree with hipcc for gfx950 (no JIT cache: the .so
travels to the GPU box with the repo snapshot)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# ORCG_PHASE_PROF=1 builds the phase-profiling variant (kernel cycle counters,
# scripts/phase_prof.py) as liborcgpu_prof.so next to the product library.
PROF = os.environ.get("ORCG_PHASE_PROF", "") == "1"
# ORCG_AB=1 builds the A/B variant (the device copy probes of
# probe_kernels.hip, scripts/ab_rlev2.py --refs probe5) as liborcgpu_ab.so.
AB = os.environ.get("ORCG_AB", "") == "1"
OUT = os.path.join(HERE, "liborcgpu_prof.so" if PROF else ("liborcgpu_ab.so" if AB else "liborcgpu.so"))
OBJ = os.path.join(HERE, "build_prof" if PROF else ("build_ab" if AB else "build"))
ARCH = os.environ.get("ORCG_OFFLOAD_ARCH", "gfx950")

SOURCES = ["rlev2_kernels.hip", "rlev2_tiled.hip", "rlev2_expand.hip", "byterle_kernels.hip", "column_kernels.hip", "rlev1_kernels.hip", "decimal_kernels.hip", "orcg_api.cpp", "rlev1_api.cpp", "orc_file.cpp", "reader_api.cpp", "byterle_api.cpp", "decimal_api.cpp", "encoder.cpp", "java_face.cpp"]
if PROF or AB:
    SOURCES.append("probe_kernels.hip")
HEADERS = ["orcg_internal.hh", "rlev2_device.hh", "orc_file.hh", os.path.join("..", "..", "include", "orcg.h"),
           os.path.join("..", "..", "include", "orcg_reader.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-Wno-unused-result", "-Wno-unused-value"]
if PROF:
    FLAGS.append("-DORCG_PHASE_PROF")
if PROF or AB:
    # experiment knobs of the A/B build (e.g. ORCG_AB_FLAGS="-DORCG_ITEM_MAX=1")
    FLAGS.extend(os.environ.get("ORCG_AB_FLAGS", "").split())


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


def build(force=False, verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    hdr_time = max(_mtime(os.path.join(CSRC, h)) for h in HEADERS)
    objs, cmds = [], []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OBJ, s + ".o")
        objs.append(obj)
        if not force and _mtime(obj) > max(_mtime(src), hdr_time):
            continue
        cmd = [HIPCC] + FLAGS + ["-c", src, "-o", obj]
        if s.endswith(".hip"):
            cmd[1:1] = ["-x", "hip", "--offload-arch=" + ARCH]
        else:
            cmd[1:1] = ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
        cmds.append(cmd)
    # translation units compile in parallel (the slowest, rlev2_tiled.hip, first)
    cmds.sort(key=lambda c: "rlev2_tiled" not in c[-3])
    from concurrent.futures import ThreadPoolExecutor

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)

    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", "8") or 8), os.cpu_count() or 1))
    with ThreadPoolExecutor(jobs) as ex:
        for f in [ex.submit(run, c) for c in cmds]:
            f.result()
    if force or _mtime(OUT) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", "-o", OUT] + objs + ["-Wl,-soname," + os.path.basename(OUT), "-lz", "-ldl", "-lpthread"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
