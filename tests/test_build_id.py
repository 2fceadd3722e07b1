"""Build provenance: the in-tree HIP library carries the hash of the sources it was built from
(gpmpc_build_id, Makefile HASHED); it must equal the hash of this tree's sources, so a stale library or
an A/B variant left in its place is refused instead of measured.  The CPU test runs here (the
library loads without a GPU); the GPU test repeats the check in the process that runs the kernels."""

import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _info():
    from gpmpc import _lib

    if not _lib.LIB_PATH.exists():
        pytest.skip("library not built (run __graft_entry__.build())")
    return _lib.build_info()


def test_library_source_hash_matches_tree():
    info = _info()
    assert info["matches_tree"], info
    assert "kind=product" in info["build_id"], info


def test_build_commit_is_an_ancestor_of_head():
    """Informational git field: the commit the library was built at is this checkout's HEAD or an
    ancestor of it (the sources may be committed after the build; the source hash above is the
    binding check).  Skipped where there is no .git (the GPU box gets the tree without it)."""
    info = _info()
    head = info["build_id"].split("git=")[1].split()[0].split("+")[0]
    if head == "nogit" or not (ROOT / ".git").exists():
        pytest.skip("no git checkout")
    r = subprocess.run(["git", "-C", str(ROOT), "merge-base", "--is-ancestor", head, "HEAD"], capture_output=True)
    assert r.returncode == 0, (head, r.stderr)


@pytest.mark.gpu
def test_gpu_process_runs_the_tree_library():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gpmpc import _lib

    _lib.load()   # refuses a library whose source hash differs from the tree's
    info = _info()
    print("build:", info)
    assert info["matches_tree"], info
