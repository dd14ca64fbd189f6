"""Run a reference entry script (run_random_sampling.py, run_BM25_negative.py, ...)
unchanged with the hot path served by this build:

    python -m denseretrievaltoolkits_amd.run path/to/run_random_sampling.py <script args>
    torchrun --nproc-per-node 8 -m denseretrievaltoolkits_amd.run run_random_sampling.py ...
"""
import os
import runpy
import sys


def main():
    if len(sys.argv) < 2:
        print(__doc__)
        sys.exit(2)
    script = sys.argv[1]
    sys.argv = sys.argv[1:]
    sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
    from . import drt_overlay
    drt_overlay.install()
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
