"""TEST INFRASTRUCTURE ONLY: compile oracle/oracle.c into oracle/_build/liboracle.so and the
OpenMP CPU-baseline kernels oracle/omp_cycle.c into oracle/_build/libomp_cycle.so (gcc)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_build", "liboracle.so")
OUT_OMP = os.path.join(HERE, "_build", "libomp_cycle.so")


def build(verbose=False):
    src = os.path.join(HERE, "oracle.c")
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= os.path.getmtime(src):
        return OUT
    cmd = ["gcc", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math", "-std=c11",
           src, "-o", OUT + ".tmp", "-lm"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


def build_omp(verbose=False):
    """No -march=native: the library is built here and run on the GPU box's host."""
    src = os.path.join(HERE, "omp_cycle.c")
    os.makedirs(os.path.dirname(OUT_OMP), exist_ok=True)
    if os.path.exists(OUT_OMP) and os.path.getmtime(OUT_OMP) >= os.path.getmtime(src):
        return OUT_OMP
    cmd = ["gcc", "-O3", "-fopenmp", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
           "-std=c11", src, "-o", OUT_OMP + ".tmp", "-lm"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT_OMP + ".tmp", OUT_OMP)
    return OUT_OMP


if __name__ == "__main__":
    print(build(True))
    print(build_omp(True))
