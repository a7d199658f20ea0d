"""ORACLE package: CPU restatements of the reference path, test infrastructure only.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg - never from fac_fake_amd (the product path has no CPU
fallback).  Pinned by reference-generated goldens under tests/golden/
(tools/make_golden.py imports CViT-main/model/cvit.py in the build container).
"""
