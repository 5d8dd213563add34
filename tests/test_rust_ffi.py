"""The Rust FFI crate (rust/omr-gpu-sys) against the C header it binds (include/omr_gpu.h).

cargo/rustc are absent from this image, so the crate cannot be built here; this check stands in
for the build: every function the header declares has exactly one `extern "C"` declaration in
src/lib.rs with the same name, the same number of parameters and the same pointer / value shape
per parameter, and the crate declares nothing the header does not. The #[repr(C)] structs carry
the header's fields in order."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "omr_gpu.h")
LIB = os.path.join(ROOT, "rust", "omr-gpu-sys", "src", "lib.rs")


def _split_params(s):
    s = s.strip()
    if s in ("", "void"):
        return []
    return [p.strip() for p in s.split(",")]


def header_functions():
    text = re.sub(r"/\*.*?\*/", " ", open(HDR).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b[\w\s\*]+?\b(omr_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text):
        params = _split_params(m.group(2))
        out[m.group(1)] = ["ptr" if "*" in p or "[" in p else "val" for p in params]
    return out


def rust_functions():
    text = open(LIB).read()
    block = text[text.index('extern "C" {'):]
    block = block[:block.index("\n    }\n")]
    block = re.sub(r"//[^\n]*", " ", block)
    out = {}
    for m in re.finditer(r"pub fn (omr_[a-z0-9_]+)\s*\((.*?)\)\s*(->\s*[^;]+)?;", block, flags=re.S):
        assert m.group(1) not in out, f"duplicate declaration {m.group(1)}"
        params = _split_params(m.group(2))
        out[m.group(1)] = ["ptr" if "*mut" in p or "*const" in p else "val" for p in params]
    return out


def test_every_header_function_bound_with_same_shape():
    h, r = header_functions(), rust_functions()
    assert len(h) >= 30, sorted(h)
    assert set(h) == set(r), f"header only {sorted(set(h) - set(r))}, crate only {sorted(set(r) - set(h))}"
    for name in sorted(h):
        assert h[name] == r[name], f"{name}: header {h[name]} vs crate {r[name]}"


@pytest.mark.parametrize("c_name,rust_name", [("omr_retrieval_params", "OmrRetrievalParams"),
                                              ("omr_detection_key_view", "OmrDetectionKeyView"),
                                              ("omr_detect_timing", "OmrDetectTiming")])
def test_repr_c_structs_match_header(c_name, rust_name):
    text = re.sub(r"/\*.*?\*/", " ", open(HDR).read(), flags=re.S)
    body = re.search(r"typedef struct \{([^{}]*)\}\s*" + c_name + ";", text).group(1)
    c_fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        names = decl.split(None, 1)[1] if not decl.startswith("const") else decl.split(None, 2)[2]
        c_fields += [n.strip().lstrip("*").strip() for n in names.split(",")]
    rs = open(LIB).read()
    rbody = re.search(r"pub struct " + rust_name + r" \{(.*?)\}", rs, flags=re.S).group(1)
    r_fields = re.findall(r"pub (\w+):", rbody)
    assert c_fields == r_fields


def test_crate_layout_and_link_directives():
    crate = os.path.join(ROOT, "rust", "omr-gpu-sys")
    toml = open(os.path.join(crate, "Cargo.toml")).read()
    assert 'links = "omr_gpu"' in toml and 'name = "omr-gpu-sys"' in toml
    build = open(os.path.join(crate, "build.rs")).read()
    assert "rustc-link-lib=dylib=omr_gpu" in build
    lib = open(LIB).read()
    for api in ("pub fn detect(", "pub fn detect_batch(", "pub fn encode_pertinent_indices(",
                "pub fn encode_pertinent_payloads(", "pub fn detect_with_time_info(", "pub fn decode_digest("):
        assert api in lib, api


def test_detect_time_info_mirrors_reference_struct():
    """DetectTimeInfo carries the reference struct's fields in its order (detector.rs:51-57:
    total_detect_time, total_first_level_bootstrapping_time, total_second_level_bootstrapping_time,
    total_trace_time), as Durations converted from omr_detect_timing."""
    rs = open(LIB).read()
    body = re.search(r"pub struct DetectTimeInfo \{(.*?)\n\}", rs, flags=re.S).group(1)
    assert re.findall(r"pub (\w+): Duration", body) == [
        "total_detect_time", "total_first_level_bootstrapping_time", "total_second_level_bootstrapping_time",
        "total_trace_time"]
    conv = re.search(r"impl From<OmrDetectTiming> for DetectTimeInfo \{(.*?)\n\}", rs, flags=re.S).group(1)
    for rust_f, c_f in (("total_detect_time", "total_ms"), ("total_first_level_bootstrapping_time", "first_level_ms"),
                        ("total_second_level_bootstrapping_time", "second_level_ms"), ("total_trace_time", "trace_ms")):
        assert re.search(rust_f + r": ms\(t\." + c_f + r"\)", conv), rust_f
    # detect_with_time_info is one locked C call, not an enable / detect / read / disable sequence
    dwt = re.search(r"pub fn detect_with_time_info\(.*?\n    \}", rs, flags=re.S).group(0)
    assert "omr_detect_with_time_info(" in dwt and "omr_ctx_enable_timing" not in dwt


def test_decode_digest_uses_board_combination_count():
    """Retriever::decode_digest regenerates the weights with the board's RetrievalParams and solves
    with its combination count (retriever.rs:196, :215-239), not a count derived from the indices
    found."""
    rs = open(LIB).read()
    dd = re.search(r"pub fn decode_digest\(.*?\n    \}", rs, flags=re.S).group(0)
    assert "payload_weights(seed, &rp)" in dd and "rp.layout.combination_count" in dd
    assert "RetrievalParams::new" not in dd
