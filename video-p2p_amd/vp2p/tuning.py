"""Library-kernel selection recorded offline for the MI355X (no tuning at run time).

Convolutions run on MIOpen.  ``miopen_db/`` holds MIOpen's user find/perf database for every
convolution shape the pipeline runs, tuned on the MI355X by tools/miopen_tune.py
(MIOPEN_FIND_ENFORCE=3: each solver's kernel parameters searched, the fastest recorded).  MIOpen
reads ``MIOPEN_USER_DB_PATH`` when it initialises, so ``use_tuned_libraries()`` must run before the
first convolution; immediate mode then takes the recorded solver of every shape instead of its
heuristic, with no search at run time.  ``miopen_db/kcache`` holds MIOpen's compiled-kernel cache for
those convolutions (MIOPEN_CUSTOM_CACHE_DIR; written by a run on the MI355X, tools/miopen_cache.sh),
so a fresh box does not compile them again -- the fp32 path (every convolution on MIOpen) at 24
frames otherwise spends minutes compiling.

(PyTorch TunableOp was tried for the GEMMs and rejected: its cold-cache timings picked solutions
slower than hipBLASLt's own heuristic in the warm pipeline, 2.53 vs 2.46 s per edit.)
"""
from __future__ import annotations

import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MIOPEN_DB = os.path.join(ROOT, "miopen_db")
MIOPEN_KCACHE = os.path.join(MIOPEN_DB, "kcache")


def use_tuned_libraries() -> dict:
    """Point MIOpen at the in-tree database and kernel cache (unless the caller chose others)."""
    used = {}
    if os.path.isdir(MIOPEN_DB):
        os.environ.setdefault("MIOPEN_USER_DB_PATH", MIOPEN_DB)
        used["miopen_db"] = os.environ["MIOPEN_USER_DB_PATH"]
    if os.path.isdir(MIOPEN_KCACHE):
        os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", MIOPEN_KCACHE)
        used["miopen_kcache"] = os.environ["MIOPEN_CUSTOM_CACHE_DIR"]
    return used
