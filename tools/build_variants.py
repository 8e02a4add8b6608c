"""Build A/B variants of libtriad_hip.so with different compile-time knobs into
tools/variants/lib_<name>.so (each with its own object dir). Load one with
TRIAD_LIB_VARIANT=<path> (triad_amd/_lib.py). Experiments only; the product build is
triad_amd/build.py with the defaults.

usage: python tools/build_variants.py name1="-DKNOB=1 -DOTHER=2" name2="..."
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(specs):
    out = os.path.join(ROOT, "tools", "variants")
    os.makedirs(out, exist_ok=True)
    for spec in specs:
        name, flags = spec.split("=", 1)
        env = dict(os.environ, TRIAD_LIB_OUT=os.path.join(out, f"lib_{name}.so"),
                   TRIAD_OBJ_DIR=os.path.join(out, f"obj_{name}"), TRIAD_EXTRA_FLAGS=flags)
        subprocess.run([sys.executable, os.path.join(ROOT, "triad_amd", "build.py")], env=env, check=True)
        print("built", name, flags)


if __name__ == "__main__":
    main(sys.argv[1:])
