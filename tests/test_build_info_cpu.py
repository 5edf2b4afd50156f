"""Build provenance stamp (neuronabox-nccl_amd/lib/build_info.json): build()
writes it, the bench line and smoke() report it. CPU only."""
import json
import os
import shutil

import pytest


def test_source_digest_tracks_content_and_names(nbx, tmp_path):
    csrc, inc = tmp_path / "csrc", tmp_path / "include"
    shutil.copytree(nbx.CSRC_DIR, csrc, ignore=shutil.ignore_patterns("*.o", "__pycache__"))
    shutil.copytree(nbx.INCLUDE_DIR, inc)
    d0, n0 = nbx.source_digest(str(csrc), str(inc))
    assert (d0, n0) == nbx.source_digest(nbx.CSRC_DIR, nbx.INCLUDE_DIR)
    assert n0 >= 30
    with open(csrc / "nbx_simple.h", "a") as f:       # one byte more in one kernel header
        f.write("\n")
    d1, n1 = nbx.source_digest(str(csrc), str(inc))
    assert n1 == n0 and d1 != d0
    os.rename(csrc / "nbx_simple.h", csrc / "nbx_simple2.h")   # same bytes, another name
    assert nbx.source_digest(str(csrc), str(inc))[0] not in (d0, d1)
    (csrc / "notes.txt").write_text("not a source")            # non-sources are ignored
    (csrc / "nbx_simple2.h").rename(csrc / "nbx_simple.h")
    assert nbx.source_digest(str(csrc), str(inc))[0] == d1


def test_build_info_flags_a_foreign_library(nbx, tmp_path):
    if not os.path.exists(nbx.library_path()):
        pytest.skip("library not built")
    p = tmp_path / "build_info.json"
    rec = nbx.write_build_info(str(p))
    assert rec["lib_bytes"] == os.path.getsize(nbx.library_path()) and rec["arch"] == "gfx950"
    assert nbx.build_info(str(p)) == {"recorded": rec, "lib_matches": True, "sources_match": True}
    p.write_text(json.dumps(dict(rec, lib_sha256="0" * 64, sources_sha256="1" * 64)))
    bi = nbx.build_info(str(p))
    assert bi["lib_matches"] is False and bi["sources_match"] is False
    assert nbx.build_info(str(tmp_path / "absent.json"))["recorded"] is None


def test_in_tree_stamp_is_current(nbx):
    """The library in the tree is the build of the sources in the tree (build()
    restamps after every make; a plain `make` leaves the stamp behind)."""
    if not os.path.exists(nbx.BUILD_INFO_PATH):
        pytest.skip("no build stamp (build() has not run in this tree)")
    bi = nbx.build_info()
    assert bi["lib_matches"], "lib/libnbxccl.so is not the stamped build: run __graft_entry__.build()"
    assert bi["sources_match"], "sources changed since the stamped build: run __graft_entry__.build()"
