"""Library-kernel selection recorded offline for the MI355X (no tuning at run time).

Convolutions run on MIOpen.  ``miopen_db/`` holds MIOpen's user find/perf database for every
convolution shape the pipeline runs, tuned on the MI355X by tools/miopen_tune.py
(MIOPEN_FIND_ENFORCE=3: each solver's kernel parameters searched, the fastest recorded).  MIOpen
reads ``MIOPEN_USER_DB_PATH`` when it initialises, so ``use_tuned_libraries()`` must run before the
first convolution; immediate mode then takes the recorded solver of every shape instead of its
heuristic, with no search at run time.  ``miopen_db/kcache`` holds MIOpen's compiled-kernel cache for
those convolutions (MIOPEN_CUSTOM_CACHE_DIR; written by a run on the MI355X, tools/miopen_cache.sh),
so a fresh box does not compile them again -- the fp32 path (every convolution on MIOpen) at 24
frames otherwise spends minutes compiling.  MIOpen is pointed at a per-user copy of both
(``seeded_cache_dir``), never at the tracked files.

(PyTorch TunableOp was tried for the GEMMs and rejected: its cold-cache timings picked solutions
slower than hipBLASLt's own heuristic in the warm pipeline, 2.53 vs 2.46 s per edit.)
"""
from __future__ import annotations

import hashlib
import os
import shutil
import tempfile
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MIOPEN_DB = os.path.join(ROOT, "miopen_db")
MIOPEN_KCACHE = os.path.join(MIOPEN_DB, "kcache")


def _seed_files():
    out = []
    for d, sub in ((MIOPEN_DB, ""), (MIOPEN_KCACHE, "kcache")):
        if os.path.isdir(d):
            out += [(os.path.join(d, n), os.path.join(sub, n)) for n in sorted(os.listdir(d))
                    if n.endswith((".txt", ".ukdb")) and os.path.isfile(os.path.join(d, n))]
    return out


def seeded_cache_dir() -> str:
    """A per-user, writable copy of the in-tree MIOpen database and kernel cache.  MIOpen writes
    into both (a new shape's find result, a newly compiled kernel), so pointing it at the tracked
    files would modify the checkout and fail on a read-only one.  The copy is keyed by the in-tree
    files' content: a changed database gets a fresh copy, the committed files are never written."""
    files = _seed_files()
    # keyed by name, size and mtime (not a hash of every byte: the kernel cache is tens of MB and
    # every rank of every process start would read it)
    h = hashlib.sha1()
    for src, rel in files:
        st = os.stat(src)
        h.update(f"{rel}:{st.st_size}:{st.st_mtime_ns}".encode())
    base = os.environ.get("XDG_CACHE_HOME") or os.path.join(os.path.expanduser("~"), ".cache")
    try:
        os.makedirs(base, exist_ok=True)
        if not os.access(base, os.W_OK):
            raise OSError(base)
    except OSError:
        base = tempfile.gettempdir()
    dst = os.path.join(base, "vp2p", f"miopen-{h.hexdigest()[:12]}")
    if not os.path.isdir(dst):
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        tmp = tempfile.mkdtemp(prefix="seed-", dir=os.path.dirname(dst))
        os.makedirs(os.path.join(tmp, "kcache"), exist_ok=True)
        for src, rel in files:
            shutil.copy2(src, os.path.join(tmp, rel))
        try:
            os.rename(tmp, dst)          # atomic; a concurrent process may have won the race
        except OSError as e:
            if os.path.isdir(dst):       # lost the race: the winner's copy is the same content
                shutil.rmtree(tmp, ignore_errors=True)
            else:                        # EXDEV, permissions, ...: keep using the private copy
                warnings.warn(f"vp2p.tuning: could not publish the MIOpen seed copy at {dst} ({e}); "
                              f"using {tmp}")
                return tmp
    if not os.path.isdir(dst):
        raise RuntimeError(f"vp2p.tuning: MIOpen seed directory {dst} is missing")
    return dst


def use_tuned_libraries() -> dict:
    """Point MIOpen at a writable copy of the in-tree database and kernel cache (unless the caller
    chose others)."""
    used = {}
    if not _seed_files():
        return used
    if "MIOPEN_USER_DB_PATH" not in os.environ or "MIOPEN_CUSTOM_CACHE_DIR" not in os.environ:
        d = seeded_cache_dir()
        os.environ.setdefault("MIOPEN_USER_DB_PATH", d)
        os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(d, "kcache"))
    used["miopen_db"] = os.environ["MIOPEN_USER_DB_PATH"]
    used["miopen_kcache"] = os.environ["MIOPEN_CUSTOM_CACHE_DIR"]
    return used
