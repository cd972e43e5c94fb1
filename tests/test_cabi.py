"""The C-ABI library loads without a GPU and exports every symbol include/sme.h
declares (no compute calls here)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "sme.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sme_[a-z_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for must in ("sme_create", "sme_build_index", "sme_build_index_device", "sme_query_topk",
                 "sme_index_partition_records", "sme_tokenize", "sme_load_docno_mapping"):
        assert must in syms


def test_library_exports_all(sme):
    L = sme.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert set(declared_symbols()) <= set(sme.EXPORTS) | {"sme_synth_corpus", "sme_synth_free"}


def test_no_gpu_fails_loudly(sme):
    import torch
    if torch.cuda.is_available():
        return
    try:
        sme.Context()
    except sme.SmeError as e:
        assert e.code < 0
    else:
        raise AssertionError("context creation must fail without a GPU (no CPU fallback)")
