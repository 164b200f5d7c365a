#!/usr/bin/env python
"""Development A/B builds (never the product): variant libraries for scripts/ab_tpch.sh.

Each variant recompiles sparksched.hip and the bench-shape translation unit (k_bench900.hip) with its own
defines and links them with the in-tree objects of the other translation units (build/obj, from
`python __graft_entry__.py build`), so a variant costs one ~1 min compile instead of a full build. Only the
bench shape (10 executors, 50 jobs, stage cap 900) is meant to run on a variant.

usage: python scripts/build_ab.py name=-DFOO=1,-DBAR name2= name3@/path/to/csrc= ...
  (an empty define list = the current sources; `@dir` compiles that directory's sources instead, e.g. a
   `git show HEAD:...` export of the previous version for a before/after comparison)
Writes gym-sparksched_amd/build/ab/<name>.so (the directory is emptied first).
"""

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

AB = os.path.join(G.BUILD, os.environ.get("AB_OUT", "ab"))  # AB_OUT: another variant directory
# translation units recompiled per variant (AB_TUS, comma-separated; default: the ABI + the bench-shape kernels)
VARIANT_TUS = tuple(os.environ.get("AB_TUS", "sparksched.hip,k_bench900.hip").split(","))


def build_variant(name, defines):
    name, _, csrc = name.partition("@")
    csrc = csrc or G.CSRC
    objdir = os.path.join(AB, "obj_" + name)
    os.makedirs(objdir, exist_ok=True)
    objs = []
    for tu in VARIANT_TUS:
        obj = os.path.join(objdir, tu + ".o")
        subprocess.run([G._hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *(G.SCHED_FLAGS if tu in G.SCHED_TUS else []), *defines,
                        f"-I{os.path.join(REPO, 'include')}", f"-I{csrc}", "-c", os.path.join(csrc, tu), "-o",
                        obj], check=True)
        objs.append(obj)
    base = [os.path.join(G.BUILD, "obj", os.path.basename(s) + ".o") for s in G.HIP_SOURCES
            if os.path.basename(s) not in VARIANT_TUS]
    out = os.path.join(AB, name + ".so")
    subprocess.run([G._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, *base, "-o", out], check=True)
    shutil.rmtree(objdir)
    return out


def main():
    shutil.rmtree(AB, ignore_errors=True)
    os.makedirs(AB)
    specs = []
    for a in sys.argv[1:]:
        name, _, defs = a.partition("=")
        specs.append((name, [d for d in defs.split(",") if d]))
    with ThreadPoolExecutor(len(specs)) as ex:
        for out in ex.map(lambda s: build_variant(*s), specs):
            print("built", out)


if __name__ == "__main__":
    main()
