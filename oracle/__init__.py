"""ORACLE — CPU restatement of MultimodalStudio's per-ray training hot path (test infrastructure).

This package is the parity checker.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it; the product package ``multimodalstudio_amd`` never does.

Every function cites the reference file:line it restates (paths relative to /root/reference).
It is pinned against golden vectors produced by running the reference itself in the build
container (tests/golden/make_golden.py -> tests/golden/*.npz).
"""
