"""Build an A/B variant of the HIP library: pokegym_amd/lib/libpokegym_amd_<name>.so.

usage: python tools/build_variant.py NAME [--rev GITREV] [-- extra hipcc flags]
--rev builds the csrc/ and include/ of a git revision (e.g. HEAD for the committed kernel) instead
of the working tree; extra flags (e.g. -DPK_SOMETHING=1) go to every compile."""
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from pokegym_amd import build as B  # noqa: E402


def main():
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        k = args.index("--")
        args, extra = args[:k], args[k + 1:]
    name = args[0]
    rev = args[args.index("--rev") + 1] if "--rev" in args else None
    out = os.path.join(B.LIBDIR, f"libpokegym_amd_{name}.so")
    if rev is None:
        print(B.build(out=out, extra=extra))
        return
    with tempfile.TemporaryDirectory() as td:
        for sub in ("pokegym_amd/csrc", "include"):
            os.makedirs(os.path.join(td, sub), exist_ok=True)
            files = subprocess.run(["git", "-C", HERE, "ls-tree", "--name-only", f"{rev}:{sub}"], check=True,
                                   capture_output=True, text=True).stdout.split()
            for f in files:
                data = subprocess.run(["git", "-C", HERE, "show", f"{rev}:{sub}/{f}"], check=True,
                                      capture_output=True).stdout
                open(os.path.join(td, sub, f), "wb").write(data)
        csrc = os.path.join(td, "pokegym_amd", "csrc")
        objs = []
        units = [(src, os.path.splitext(src)[0], []) for src in B.SOURCES]
        if "PK_K1_SMALL" in open(os.path.join(td, "pokegym_amd", "csrc", "pk_step.hip")).read():
            units.append(("pk_step.hip", "pk_step_small", ["-DPK_K1_SMALL"]))
        for src, stem, defs in units:
            obj = os.path.join(td, stem + ".o")
            cmd = [B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-w", "-c", "-o", obj] + defs + extra
            if src.endswith(".cpp"):
                cmd += ["-x", "hip"]
            subprocess.run(cmd + [os.path.join(csrc, src)], check=True)
            objs.append(obj)
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out] + objs, check=True)
    print(out)


if __name__ == "__main__":
    main()
