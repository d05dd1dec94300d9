#!/usr/bin/env python3
"""Builds an A/B variant of the product library from a patched copy of the sources (the product
tree is untouched): each SUB is FILE:OLD=>NEW, an exact one-time replacement in csrc/FILE.  The
library goes to OUT (use it with FRAC_LIB=OUT in tools/bench_paths.py; bench.py refuses a foreign
library for its headline).
usage: tools/build_variant.py [--git REV] OUT.so 'fracenc_api.hip:old text=>new text' [...]"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402

args = sys.argv[1:]
rev = None
if args and args[0] == "--git":  # the sources of a committed revision instead of the working tree
    rev, args = args[1], args[2:]
out = os.path.abspath(args[0])
with tempfile.TemporaryDirectory() as d:
    pkg = os.path.join(d, "fractencode_amd")
    shutil.copytree(G.CSRC, os.path.join(pkg, "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(d, "include"))
    if rev:
        for sub_dir, dst in (("fractencode_amd/csrc", os.path.join(pkg, "csrc")), ("include", os.path.join(d, "include"))):
            names = subprocess.check_output(["git", "ls-tree", "--name-only", rev, sub_dir + "/"], cwd=ROOT, text=True).split()
            for name in names:
                data = subprocess.check_output(["git", "show", f"{rev}:{name}"], cwd=ROOT)
                open(os.path.join(dst, os.path.basename(name)), "wb").write(data)
    for sub in args[1:]:
        fname, rest = sub.split(":", 1)
        old, new = rest.split("=>", 1)
        path = os.path.join(pkg, "csrc", fname)
        text = open(path).read()
        if text.count(old) != 1:
            sys.exit(f"{fname}: '{old}' occurs {text.count(old)} times (need exactly 1)")
        open(path, "w").write(text.replace(old, new))
    cmd = G.hipcc_cmd(out, "-DFRAC_AB_VARIANT")
    cmd[-1] = os.path.join(pkg, "csrc", "fracenc_api.hip")
    subprocess.check_call(cmd, cwd=os.path.join(pkg, "csrc"))
print(out)
