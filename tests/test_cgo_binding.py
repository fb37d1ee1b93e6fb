"""The cgo package (internal/hipquorum/*.go) against the C-ABI it binds (include/hipquorum.h).

No Go toolchain exists in this image, so the Go side cannot be compiled here. This test pins it
to the header mechanically: every C.hq_* function call names a declared function with the
declared number of arguments, every C.HQ_* constant is #defined, every C.hq_* type exists,
every field of a C struct composite literal and every field selected through an identifier of a
known C struct type is a field of that struct, and the package checks the library's ABI version
when it opens (VERDICT r04 "internal/hipquorum as a file")."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hipquorum.h")
PKG = os.path.join(ROOT, "internal", "hipquorum")
GO_KEYWORDS = {"type", "func", "range", "map", "chan", "go", "select", "default", "var"}
# cgo pseudo-functions and C types used as conversions
CGO_BUILTINS = {"GoString", "GoStringN", "GoBytes", "CString", "CBytes", "malloc", "calloc", "free"}
C_SCALARS = {"int", "uint", "char", "uchar", "size_t", "double", "float", "uint8_t", "uint16_t",
             "uint32_t", "uint64_t", "int8_t", "int16_t", "int32_t", "int64_t", "uintptr_t"}


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _split_top(args):
    """Top-level comma split of an argument text (parentheses, brackets and braces nest)."""
    out, depth, cur = [], 0, ""
    for ch in args:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [a.strip() for a in out if a.strip()]


def parse_header():
    s = _strip_c_comments(open(HEADER).read())
    funcs = {}
    for m in re.finditer(r"\b(?:static\s+inline\s+)?(?:const\s+)?(?:int|void|char|uint32_t|uint64_t|"
                         r"size_t)\s*\*?\s*(hq_\w+)\s*\(([^;{]*?)\)\s*[;{]", s, flags=re.S):
        args = " ".join(m.group(2).split())
        funcs[m.group(1)] = 0 if args in ("", "void") else len(_split_top(args))
    consts = set(re.findall(r"^\s*#define\s+(HQ_\w+)", s, flags=re.M))
    structs = {}
    for m in re.finditer(r"typedef\s+struct\s+(hq_\w+)\s*\{(.*?)\}\s*(hq_\w+)\s*;", s, flags=re.S):
        fields = set()
        for decl in m.group(2).split(";"):
            decl = decl.strip()
            if not decl:
                continue
            # "type a, *b, c[4]": the declarators after the type
            parts = _split_top(decl)
            first = re.match(r"^(.*?)(\**\s*\w+\s*(\[[^\]]*\])?)$", parts[0])
            decls = [first.group(2)] + parts[1:]
            for dcl in decls:
                name = re.sub(r"\[.*\]", "", dcl).strip().lstrip("*").strip()
                fields.add(name)
        structs[m.group(3)] = fields
    opaque = set(re.findall(r"typedef\s+struct\s+(hq_\w+)\s+(hq_\w+)\s*;", s))
    types = set(structs) | {b for _, b in opaque}
    return funcs, consts, structs, types


def go_sources():
    files = sorted(f for f in os.listdir(PKG) if f.endswith(".go"))
    return {f: open(os.path.join(PKG, f)).read() for f in files}


def _strip_go(s):
    s = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), s, flags=re.S)
    s = re.sub(r"//[^\n]*", "", s)
    return re.sub(r'"(\\.|[^"\\])*"', '""', s)


def _calls(src):
    """(name, argument text) of every C.name( ... ) in src, the parentheses matched."""
    for m in re.finditer(r"\bC\.(\w+)\(", src):
        i, depth = m.end(), 1
        while depth:
            ch = src[i]
            depth += ch == "("
            depth -= ch == ")"
            i += 1
        yield m.group(1), src[m.end():i - 1], m.start()


def _composites(src):
    """(type, body) of every C.hq_T{ ... } composite literal."""
    for m in re.finditer(r"\bC\.(hq_\w+)\{", src):
        i, depth = m.end(), 1
        while depth:
            ch = src[i]
            depth += ch == "{"
            depth -= ch == "}"
            i += 1
        yield m.group(1), src[m.end():i - 1]


def _functions(src):
    """Top-level declarations split at each 'func ' at column 0 (a scope per function)."""
    parts = re.split(r"(?m)^func ", src)
    return parts[0], ["func " + p for p in parts[1:]]


def _typed_idents(text):
    """identifier -> C struct type for declarations in text: `x *C.hq_T`, `x C.hq_T` (params,
    results, struct fields, var), `x := C.hq_T{`, `x := unsafe.Slice((*C.hq_T)(...` and
    `x = (*C.hq_T)(...` assignments."""
    out = {}
    for m in re.finditer(r"\b(\w+)\s+\*?C\.(hq_\w+)\b", text):
        out[m.group(1)] = m.group(2)
    for m in re.finditer(r"\b(\w+)\s*:?=\s*(?:&)?C\.(hq_\w+)\{", text):
        out[m.group(1)] = m.group(2)
    for m in re.finditer(r"\b(\w+)\s*:?=\s*unsafe\.Slice\(\(\*C\.(hq_\w+)\)", text):
        out[m.group(1)] = m.group(2)
    return out


@pytest.fixture(scope="module")
def header():
    return parse_header()


def test_package_files_exist():
    src = go_sources()
    assert {"hipquorum.go", "engine.go", "worker.go"} <= set(src)
    for f, s in src.items():
        assert re.search(r"(?m)^package hipquorum$", s), f
        assert 'import "C"' in s and '#include "hipquorum.h"' in s, f


def test_preamble_and_abi_check(header):
    s = go_sources()["hipquorum.go"]
    # the cgo preamble in the reference's own style (gorocksdb/db.go:3-9): flags, then includes
    assert re.search(r"/\*\s*\n#cgo CFLAGS: -I\$\{SRCDIR\}/\.\./\.\./include\n#cgo LDFLAGS: .*-lhipquorum",
                     s)
    assert "C.hq_abi_version()" in s and "C.HQ_ABI_VERSION" in s
    # every constructor checks the ABI before its first call into the library
    src = _strip_go("\n".join(go_sources().values()))
    for fn in ("Open", "OpenWorker", "OpenDeviceWorker", "DeviceCount"):
        m = re.search(r"(?m)^func %s\(.*?\n\}" % fn, src, flags=re.S)
        assert m, fn
        body = m.group(0)
        assert body.index("checkABI()") < body.index("C.hq_"), fn


def test_every_call_matches_the_header(header):
    funcs, consts, structs, types = header
    seen = set()
    for f, raw in go_sources().items():
        src = _strip_go(raw)
        for name, args, pos in _calls(src):
            line = src.count("\n", 0, pos) + 1
            if name in CGO_BUILTINS or name in C_SCALARS:
                continue
            if name in types:          # a conversion (*C.hq_T)(p) is matched as C.hq_T)( ...
                continue
            assert name in funcs, f"{f}:{line}: C.{name} is not declared in include/hipquorum.h"
            n = len(_split_top(args))
            assert n == funcs[name], (f"{f}:{line}: C.{name} takes {funcs[name]} arguments, the "
                                      f"binding passes {n}")
            seen.add(name)
    # the package binds the hot path and its callers
    for need in ("hq_open", "hq_commit", "hq_commit_dev", "hq_commit_fused_dev", "hq_engine_post",
                 "hq_engine_wait", "hq_readindex_multi_tiles_dev",
                 "hq_readindex_vote_cq_planes_dev", "hq_worker_step_stream",
                 "hq_worker_step_jobs", "hq_events16_encode_sized_multi", "hq_worker_set_wait",
                 "hq_abi_version"):
        assert need in seen, need


def test_constants_and_types_exist(header):
    funcs, consts, structs, types = header
    for f, raw in go_sources().items():
        src = _strip_go(raw)
        for c in set(re.findall(r"\bC\.(HQ_\w+)\b", src)):
            assert c in consts, f"{f}: C.{c} is not #defined in include/hipquorum.h"
        for t in set(re.findall(r"\bC\.(hq_\w+)\b(?!\()", src)):
            assert t in types or t in funcs, f"{f}: C.{t} is not a type of include/hipquorum.h"


def test_struct_fields_exist(header):
    funcs, consts, structs, types = header

    def check(f, t, field, where):
        field = field[1:] if field.startswith("_") and field[1:] in GO_KEYWORDS else field
        assert field in structs[t], f"{f}: {where}: {field} is not a field of {t}"

    n_checked = 0
    for f, raw in go_sources().items():
        src = _strip_go(raw)
        for t, body in _composites(src):
            if t not in structs:
                continue
            for kv in _split_top(body):
                key = kv.split(":", 1)[0].strip()
                check(f, t, key, f"C.{t}{{...}}")
                n_checked += 1
        top, funcs_src = _functions(src)
        global_ids = _typed_idents(top)
        for fn in funcs_src:
            ids = dict(global_ids)
            ids.update(_typed_idents(fn))
            for m in re.finditer(r"\b(\w+)(?:\[[^\]]*\])?\.([a-z_]\w*)\b", fn):
                ident, field = m.group(1), m.group(2)
                if ident in ids and ids[ident] in structs:
                    check(f, ids[ident], field, f"{ident}.{field}")
                    n_checked += 1
    assert n_checked > 40


def test_integration_md_points_at_the_package():
    s = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "internal/hipquorum/hipquorum.go" in s and "tests/test_cgo_binding.py" in s
