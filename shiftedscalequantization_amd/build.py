"""Build libssq.so (the gfx950 HIP kernels + C ABI) in-tree with hipcc.

    python -m shiftedscalequantization_amd.build [--force]

The library lands next to this file so it travels with the repository snapshot to
the GPU box (it is git-ignored, not gpurun-ignored).  Compilation flags fix the
numerics contract: IEEE fp32 divide/sqrt, no FMA contraction.
"""
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libssq.so")
ARCH = os.environ.get("SSQ_OFFLOAD_ARCH", "gfx950")

SOURCES = ["fq.hip", "adashift.hip", "adashift_prep.hip", "scale_init.hip", "recon.hip", "pack.hip", "conv_wgrad.hip",
           "dwconv.hip", "fc_recon.hip"]
HEADERS = ["ssq_common.h", "adashift_common.h", "fin_tasks.h", "prep_ride.h", os.path.join("..", "..", "include", "ssq.h")]
CFLAGS = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-ffp-contract=off",
          "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall", "-Wno-unused-function"]


def source_sha():
    """sha256 (16 hex) of every source the library is built from (SOURCES + HEADERS, in
    that order): the provenance stamp of committed measurements (profiles/*.json), which
    bench.py compares against the tree it runs from (the GPU box has no .git)."""
    import hashlib
    h = hashlib.sha256()
    for name in SOURCES + HEADERS:
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def provenance():
    """{"csrc_sha": source_sha(), "git_sha": $SSQ_GIT_SHA or `git rev-parse HEAD` when a
    repository is present, else None}: stamped into measurement summaries."""
    sha = os.environ.get("SSQ_GIT_SHA")
    if not sha:
        try:
            sha = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], cwd=HERE,
                                 capture_output=True, text=True, timeout=10).stdout.strip() or None
        except (OSError, subprocess.SubprocessError):
            sha = None
    return {"csrc_sha": source_sha(), "git_sha": sha}


def _hipcc():
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: cannot build libssq.so")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True):
    hipcc = _hipcc()
    os.makedirs(OBJ, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS]
    jobs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src.replace(".hip", ".o"))
        if force or _stale(o, [s] + hdrs + [__file__]):
            jobs.append((s, o))

    def compile_one(job):
        s, o = job
        cmd = [hipcc] + CFLAGS + ["-c", s, "-o", o]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {s}:\n{r.stderr}")
        return s

    with cf.ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        for s in ex.map(compile_one, jobs):
            if verbose:
                print(f"[ssq build] compiled {os.path.basename(s)}")
    objs = [os.path.join(OBJ, s.replace(".hip", ".o")) for s in SOURCES]
    if force or jobs or _stale(LIB, objs):
        # link beside, then rename: a reader (or a tree snapshot) never sees a partial file
        tmp = LIB + ".tmp"
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, LIB)
        if verbose:
            print(f"[ssq build] linked {LIB}")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
