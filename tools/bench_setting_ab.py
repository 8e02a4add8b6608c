"""Run bench.py in-process with one module attribute overridden (an A/B of a product setting on
the real step), e.g.  python tools/bench_setting_ab.py triad_amd.ops.PROJHEAD_FORM=lib -- --steps 5
Alternate calls in one gpurun command to compare settings on the same box."""
import importlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv):
    i = argv.index("--") if "--" in argv else len(argv)
    sets, rest = argv[:i], argv[i + 1:]
    for s in sets:
        key, val = s.split("=", 1)
        mod, attr = key.rsplit(".", 1)
        m = importlib.import_module(mod)
        old = getattr(m, attr)
        setattr(m, attr, type(old)(val) if old is not None and not isinstance(old, str) else val)
        print(f"[setting] {key} = {getattr(m, attr)!r}", file=sys.stderr, flush=True)
    sys.argv = [os.path.join(ROOT, "bench.py")] + rest
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main(sys.argv[1:])
