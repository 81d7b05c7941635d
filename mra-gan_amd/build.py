"""Build libmragan_hip.so for gfx950 in-tree (mra-gan_amd/lib/).  No JIT cache, no torch
extension machinery: plain hipcc, one object per .hip file, parallel compile."""
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# MRAGAN_LIB_DIR / MRAGAN_OBJ_DIR / MRAGAN_EXTRA_FLAGS: variant builds for same-box A/B
# (tools/gpu_libs_ab.sh); the default is the in-tree library the package loads
LIB = os.environ.get("MRAGAN_LIB_DIR", os.path.join(HERE, "lib"))
OBJ = os.environ.get("MRAGAN_OBJ_DIR", os.path.join(HERE, "build"))
ARCH = os.environ.get("MRAGAN_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-Wno-unused-but-set-variable"] + os.environ.get("MRAGAN_EXTRA_FLAGS", "").split()


def sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))


def _needs(obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _check_no_scratch(src, remarks):
    """Every kernel must run out of registers: a private-memory (scratch) spill in an MFMA loop
    costs 20× (measured: a 2-byte/lane spill turned a 60 µs conv into 1.6 ms).  Fail the build."""
    fn = None
    bad = []
    for line in remarks.splitlines():
        if "Function Name:" in line:
            fn = line.split("Function Name:")[1].split("[")[0].strip()
        elif "ScratchSize [bytes/lane]:" in line:
            n = int(line.split("ScratchSize [bytes/lane]:")[1].split("[")[0])
            if n:
                bad.append(f"{fn}: {n} B/lane")
    if bad:
        raise RuntimeError(f"{os.path.basename(src)}: kernels use scratch (register spill): " + "; ".join(bad))


def build(verbose=False, jobs=None):
    os.makedirs(LIB, exist_ok=True)
    os.makedirs(OBJ, exist_ok=True)
    headers = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    headers.append(os.path.join(HERE, "..", "include", "mragan_hip.h"))
    objs, cmds = [], []
    for s in sources():
        src = os.path.join(CSRC, s)
        obj = os.path.join(OBJ, s.replace(".hip", ".o"))
        objs.append(obj)
        if _needs(obj, [src] + headers):
            cmds.append(["hipcc", *FLAGS, "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", obj])
    with cf.ThreadPoolExecutor(max_workers=jobs or min(8, os.cpu_count() or 1)) as ex:
        for cmd, r in zip(cmds, ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), cmds)):
            if verbose or r.returncode:
                sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
            if r.returncode:
                raise RuntimeError(f"hipcc failed for {cmd[-3]}")
            _check_no_scratch(cmd[-3], r.stderr)
    so = os.path.join(LIB, "libmragan_hip.so")
    # relink also when an object is newer than the library (an object compiled by hand for a
    # register-usage check would otherwise never reach the .so)
    if cmds or not os.path.exists(so) or any(os.path.getmtime(o) > os.path.getmtime(so) for o in objs):
        r = subprocess.run(["hipcc", "-shared", "-fPIC", f"--offload-arch={ARCH}", "-Wl,--no-undefined", *objs, "-o", so],
                           capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
    return so


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
