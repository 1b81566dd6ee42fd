#!/usr/bin/env python3
"""Build / time tuning variants of the engine (different compile-time knobs).

  python tools/ab_variants.py build NAME -DKNOB=V ...   # here (CPU), into variants/NAME.so
  python tools/ab_variants.py run                        # on the GPU box: bench every variants/*.so
"""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    if sys.argv[1] == "build":
        from charon_amd import _native
        name = sys.argv[2]
        defs = [a[2:] for a in sys.argv[3:] if a.startswith("-D")]
        print(_native.build(force=True, defines=defs, out=os.path.join(ROOT, "variants", name + ".so")))
    else:
        for so in sorted(glob.glob(os.path.join(ROOT, "variants", "*.so"))):
            env = dict(os.environ, TBG_LIB=so)
            r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "16", "--warmup", "1",
                                "--no-cpu"], env=env, capture_output=True, text=True, timeout=600)
            try:
                d = json.loads(r.stdout.strip().splitlines()[-1])
                print(os.path.basename(so), d["value"], d["kernel_ms_per_step"], flush=True)
            except Exception:
                print(os.path.basename(so), "FAILED", r.stderr[-500:], flush=True)


if __name__ == "__main__":
    main()
