"""RnB benchmark entry point (reference-compatible CLI).

    python benchmark.py -c configs/r2p1d-whole.json -v 500 -mi 90
    python benchmark.py --check

See rnb_amd/launcher.py for the flags and the process topology.
"""
import sys

if __name__ == "__main__":
    from rnb_amd.launcher import main
    sys.exit(main())
