"""The Go shim's cgo calls against include/hge.h (no Go toolchain in this image,
so this is the compile check cgo would do on the C side).

Every `C.hge_*(...)` call in go/hashgraph/*.go must name a function the header
declares, with the header's arity, and every argument whose C type can be read
off the Go source must have exactly the parameter's type (cgo's C.int32_t,
C.int64_t, C.int and C.uint8_t are distinct Go types: a mismatch does not
compile):
  * C.T(expr) conversions, and untyped constants / C.HGE_* macros (any integer);
  * nil for a pointer parameter;
  * &v and &v[0] where v is declared as `var v C.T`, `v := make([]C.T, ...)`,
    `v := []C.T{...}` or `v := C.T(...)` in the same function;
  * the engine / store handles (struct fields `*C.hge_engine`, `*C.hge_store`) and
    any struct field, map value or method result of a cgo type (`a, b := h.id(x),
    h.id(y)`, `c, err := s.creatorID(p)`, `id, ok := s.ids[key]`, `for _, v := range`);
  * (*C.T)(unsafe.Pointer(...)) casts.
Arguments of any other form (a Go variable whose type the regexes cannot see)
are listed; the test requires all but a handful to be checked.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = [os.path.join(ROOT, "go", "hashgraph", f) for f in ("hashgraph_hge.go", "inmem_store_hge.go")]


RETURNS = {}


def header_prototypes():
    src = open(os.path.join(ROOT, "include", "hge.h")).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(hge_\w+)\s*\(([^;{]*?)\)\s*;", src, flags=re.S):
        name, params = m.group(2), m.group(3).strip()
        ret = " ".join(m.group(1).replace("const ", " ").split()).split()
        RETURNS[name] = (ret[-1] if ret else "") + ""
        if params in ("", "void"):
            protos[name] = []
            continue
        types = []
        for p in params.split(","):
            p = " ".join(p.replace("const ", " ").replace("*", " * ").split())
            toks = p.split()
            if toks and toks[-1] != "*" and len(toks) > 1:
                toks = toks[:-1]  # drop the parameter name
            base = " ".join(t for t in toks if t != "*")
            types.append(base + "*" * toks.count("*"))
        protos[name] = types
    return protos


def split_args(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def go_calls(path):
    src = open(path).read()
    calls = []
    for m in re.finditer(r"C\.(hge_\w+)\(", src):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        func_start = src.rfind("\nfunc ", 0, m.start())
        calls.append((m.group(1), split_args(src[m.end():i - 1]), src[func_start:m.start()],
                      src.count("\n", 0, m.start()) + 1))
    return src, calls


def go_decls(srcs):
    """Result types of the shim's functions and types of its struct fields (Go syntax)."""
    funcs, fields = {}, {}
    for src in srcs:
        for m in re.finditer(r"\nfunc (?:\([^)]*\) )?(\w+)\(([^)]*)\)\s*([^{\n]*)\{", src):
            res = m.group(3).strip()
            if res.startswith("("):
                res = res[1:-1]
            funcs[m.group(1)] = [r.strip().split()[-1] if r.strip() else "" for r in split_args(res)] if res else []
        for m in re.finditer(r"\ntype \w+ struct \{(.*?)\n\}", src, flags=re.S):
            for line in m.group(1).splitlines():
                line = line.split("//")[0].strip()
                parts = line.split()
                if len(parts) >= 2:
                    for nm in parts[0].rstrip(",").split(","):
                        fields[nm] = parts[-1] if len(parts) > 2 and parts[0].endswith(",") else parts[1]
    return funcs, fields


def elem(t):
    """Element type of a Go slice / array / map type."""
    if t is None:
        return None
    m = re.fullmatch(r"(?:\[\d*\]|map\[[^\]]*\])(.*)", t)
    return m.group(1) if m else None


class Types:
    def __init__(self, funcs, fields):
        self.funcs, self.fields = funcs, fields

    def expr(self, e, scope):
        """Go type of an expression (as written in the source), or None."""
        e = e.strip()
        m = re.fullmatch(r"C\.(\w+)\((.*)\)", e, flags=re.S)
        if m:
            if m.group(1).startswith("hge_"):
                return "C." + RETURNS.get(m.group(1), "?")
            return "C." + m.group(1)
        m = re.fullmatch(r"(?:\w+\.)?(\w+)\((.*)\)", e, flags=re.S)
        if m and m.group(1) in self.funcs:
            r = self.funcs[m.group(1)]
            return r[0] if r else None
        m = re.fullmatch(r"\w+\.(\w+)\[(.*)\]", e, flags=re.S)
        if m and m.group(1) in self.fields:
            return elem(self.fields[m.group(1)])
        m = re.fullmatch(r"\w+\.(\w+)", e)
        if m and m.group(1) in self.fields:
            return self.fields[m.group(1)]
        m = re.fullmatch(r"(\w+)\[(.*)\]", e, flags=re.S)
        if m:
            return elem(self.var(m.group(1), scope))
        m = re.fullmatch(r"(\w+)", e)
        if m:
            return self.var(m.group(1), scope)
        return None

    def var(self, name, scope):
        """Type of the latest declaration of `name` in `scope`."""
        best = None

        def take(pos, t):
            nonlocal best
            if t is not None and (best is None or pos > best[0]):
                best = (pos, t)

        for m in re.finditer(rf"\bvar\s+((?:\w+\s*,\s*)*\w+)\s+(\S+)", scope):
            if name in [v.strip() for v in m.group(1).split(",")]:
                take(m.start(), m.group(2))
        for m in re.finditer(r"(?m)^\s*((?:\w+\s*,\s*)*\w+)\s*:?=\s*(.+)$", scope):
            lhs = [v.strip() for v in m.group(1).split(",")]
            if name not in lhs:
                continue
            k = lhs.index(name)
            rhs = split_args(m.group(2).strip())
            if len(rhs) == len(lhs):
                r = rhs[k]
                mm = re.match(r"make\((\[\][^,]+),", r)
                if mm:
                    take(m.start(), mm.group(1))
                    continue
                mm = re.match(r"(\[\]C\.\w+)\{", r)
                if mm:
                    take(m.start(), mm.group(1))
                    continue
                mm = re.match(r"(C\.\w+)\{", r)
                if mm:
                    take(m.start(), mm.group(1))
                    continue
                take(m.start(), self.expr(r, scope[:m.start()]))
            elif len(rhs) == 1:
                mm = re.fullmatch(r"(?:\w+\.)?(\w+)\((.*)\)", rhs[0], flags=re.S)
                if mm and mm.group(1) in self.funcs and k < len(self.funcs[mm.group(1)]):
                    take(m.start(), self.funcs[mm.group(1)][k])
                elif k == 0:  # v, ok := m[key]
                    take(m.start(), self.expr(rhs[0], scope[:m.start()]))
        for m in re.finditer(rf"for\s+(\w+)\s*,\s*{name}\s*:=\s*range\s+(\S+)", scope):
            take(m.start(), elem(self.expr(m.group(2), scope[:m.start()])))
        return best[1] if best else None


def c_type(t):
    """A Go type of the cgo world as the C type it stands for ('*C.int32_t' -> 'int32_t*')."""
    if t is None:
        return None
    stars = 0
    while t.startswith("*"):
        stars += 1
        t = t[1:]
    if not t.startswith("C."):
        return None
    return t[2:] + "*" * stars


def arg_type(a, scope, types):
    """C type of a Go argument expression, or None when it cannot be read off."""
    a = a.strip()
    if a == "nil":
        return "NULL"
    if re.fullmatch(r"C\.HGE_\w+|-?\d+", a):
        return "CONST"
    m = re.fullmatch(r"\(\*C\.(\w+)\)\(unsafe\.Pointer\(.*\)\)", a, flags=re.S)
    if m:
        return m.group(1) + "*"
    m = re.fullmatch(r"&(.+?)\[[^\]]*\]", a)
    if m:
        return c_type("*" + (elem(types.expr(m.group(1), scope)) or "?"))
    if a.startswith("&"):
        t = types.expr(a[1:], scope)
        return c_type("*" + t) if t else None
    return c_type(types.expr(a, scope))


INT_TYPES = {"int", "int32_t", "int64_t", "uint8_t", "int8_t", "uint32_t", "uint64_t", "size_t", "double", "float"}


def compatible(have, want):
    if have == "NULL":
        return want.endswith("*")
    if have == "CONST":
        return want in INT_TYPES
    return have == want


def test_every_call_matches_the_header():
    protos = header_prototypes()
    assert len(protos) > 80
    checked, unchecked, bad = 0, [], []
    ncalls = 0
    types = Types(*go_decls([open(p).read() for p in GO]))
    for path in GO:
        src, calls = go_calls(path)
        for name, args, scope, line in calls:
            ncalls += 1
            where = f"{os.path.basename(path)}:{line} {name}"
            assert name in protos, f"{where}: not declared in include/hge.h"
            want = protos[name]
            if len(args) != len(want):
                bad.append(f"{where}: {len(args)} arguments, hge.h declares {len(want)}")
                continue
            for k, (a, w) in enumerate(zip(args, want)):
                have = arg_type(a, scope, types)
                if have is None:
                    unchecked.append(f"{where} arg {k} `{a}` ({w})")
                    continue
                checked += 1
                if not compatible(have, w):
                    bad.append(f"{where} arg {k} `{a}`: {have}, hge.h wants {w}")
    assert ncalls >= 60
    assert not bad, "\n".join(bad)
    assert len(unchecked) <= 2, "\n".join(unchecked)


def test_checker_catches_a_mismatch():
    protos = header_prototypes()
    assert protos["hge_round_of"] == ["hge_engine*", "int32_t"]
    assert not compatible("int", "int32_t") and not compatible("int64_t", "int64_t*")
    ty = Types({"id": ["C.int32_t"], "pair": ["C.int32_t", "error"]}, {"eng": "*C.hge_engine",
                                                                       "ids": "map[string]C.int64_t"})
    assert arg_type("C.int32_t(x)", "", ty) == "int32_t"
    assert arg_type("&n", "func f() {\n var n C.int64_t\n", ty) == "int64_t*"
    assert arg_type("&ids[0]", "\n ids := make([]C.int32_t, 4)\n", ty) == "int32_t*"
    assert arg_type("h.eng", "", ty) == "hge_engine*" and arg_type("&h.eng", "", ty) == "hge_engine**"
    assert arg_type("a", "\n a, b := h.id(x), h.id(y)\n", ty) == "int32_t"
    assert arg_type("c", "\n c, err := s.pair(p)\n", ty) == "int32_t"
    assert arg_type("k", "\n k, ok := s.ids[key]\n", ty) == "int64_t"
    assert arg_type("v", "\n var w [4]C.uint8_t\n for _, v := range w {\n", ty) == "uint8_t"
