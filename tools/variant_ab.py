"""Run one micro-benchmark script against several library variants (tools/build_variants.py),
each in its own child process with TRIAD_LIB_VARIANT set, alternating the order over `rounds`
so clock drift on the box does not favour one variant.

usage: python tools/variant_ab.py <script> <rounds> default lib_a.so lib_b.so ... [-- script args]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(argv):
    script, rounds, rest = argv[0], int(argv[1]), argv[2:]
    extra = []
    if "--" in rest:
        i = rest.index("--")
        rest, extra = rest[:i], rest[i + 1:]
    libs = rest
    for r in range(rounds):
        order = libs if r % 2 == 0 else libs[::-1]
        for lib in order:
            env = dict(os.environ)
            env.pop("TRIAD_LIB_VARIANT", None)
            if lib != "default":
                env["TRIAD_LIB_VARIANT"] = os.path.join(ROOT, "tools", "variants", lib)
            rc = subprocess.run([sys.executable, os.path.join(ROOT, script)] + extra, env=env, timeout=300).returncode
            if rc != 0:
                print(f"[variant_ab] {lib} failed rc={rc}", flush=True)
                return rc
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
