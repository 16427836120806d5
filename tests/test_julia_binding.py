"""Static checks of the Julia binding (rollout-bayesian-optimization_amd/julia/MRBO.jl).

julia is not installed in this image, so the shim cannot run here.  What decides whether it can
load and bind correctly is checked from the text instead:
  * the struct mirrors MrboSurrogateC / MrboParamsC against the C structs of include/mrbo.h:
    field order, types, and byte offsets (the C offsets from gcc on the real header);
  * every `ccall` against the C prototype it names: return type, arity, argument types, and the
    number of actual arguments passed;
  * every positional struct constructor call passes one value per field;
  * scope: MRBO.jl is a `module`, which sees only Base/Core, while the reference defines its API
    at top level of `Main` (rollout_bayesian_optimization.jl:15-30 `include`s).  Every reference
    name the shim uses must come from `using Main: …` or `import Main: …`, and the generic
    functions it adds methods to (simulate_trajectory_mc rollout.jl:279, simulate_trajectory_ghq
    rollout.jl:409) must be `import`ed, or the methods would define new functions that the
    reference's call sites never reach.  The reference's names are a committed fixture
    (tests/golden/make_julia_names.py), so this test does not read /root/reference.
"""
import json
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "rollout-bayesian-optimization_amd", "julia", "MRBO.jl")
HEADER = os.path.join(ROOT, "include", "mrbo.h")
NAMES = os.path.join(ROOT, "tests", "golden", "julia_ref_names.json")
IDENT = r"[A-Za-z_¡-￿][A-Za-z0-9_!¡-￿]*"

STRUCT_MAP = {"MrboSurrogateC": "mrbo_surrogate_t", "MrboParamsC": "mrbo_params_t",
              "MrboSolveOptsC": "mrbo_solve_opts_t"}
SCALAR = {"Int32": "int32_t", "Cint": "int32_t", "UInt32": "uint32_t", "UInt64": "uint64_t", "Int64": "int64_t",
          "Float64": "double", "Cdouble": "double", "Cvoid": "void"}
SIZE_ALIGN = {"int32_t": 4, "uint32_t": 4, "int64_t": 8, "uint64_t": 8, "double": 8, "ptr": 8}


# ---------------------------------------------------------------------------------------------
# parsing helpers
def strip_julia(src):
    """Remove comments and string literals (kept as empty "")."""
    out, i, n = [], 0, len(src)
    while i < n:
        ch = src[i]
        if ch == "#":
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif ch == '"':
            j = i + 1
            while j < n and src[j] != '"':
                j += 2 if src[j] == "\\" else 1
            out.append('""')
            i = j + 1
        else:
            out.append(ch)
            i += 1
    return "".join(out)


def split_top(s):
    """Split s on commas at bracket depth 0."""
    parts, depth, cur = [], 0, []
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    if "".join(cur).strip():
        parts.append("".join(cur).strip())
    return parts


def call_body(src, open_idx):
    """Text between the parenthesis at open_idx and its match."""
    depth = 0
    for j in range(open_idx, len(src)):
        if src[j] == "(":
            depth += 1
        elif src[j] == ")":
            depth -= 1
            if depth == 0:
                return src[open_idx + 1:j]
    raise AssertionError("unbalanced parentheses")


def c_header():
    txt = open(HEADER, encoding="utf-8").read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    txt = re.sub(r"//[^\n]*", " ", txt)
    txt = re.sub(r"(?m)^\s*#.*$", " ", txt)
    structs = {}
    for body, name in re.findall(r"typedef\s+struct\s*\{(.*?)\}\s*(\w+)\s*;", txt, flags=re.S):
        fields = []
        for decl in body.split(";"):
            decl = " ".join(decl.split())
            if decl:
                m = re.match(r"(.*?)(\w+)$", decl)
                fields.append((m.group(2), canon_c(m.group(1))))
        structs[name] = fields
    protos = {}
    for chunk in re.split(r"[;{}]", txt):
        m = re.fullmatch(r"\s*([\w\s\*]+?)\b(mrbo_\w+)\s*\(([^()]*)\)\s*", chunk, flags=re.S)
        if not m or m.group(1).strip().startswith(("typedef", "#")):
            continue
        ret, name, args = m.groups()
        arglist = [] if args.strip() == "void" else [canon_c(re.match(r"(.*?)(\w+)$", " ".join(a.split())).group(1))
                                                    for a in args.split(",")]
        protos[name] = (canon_c(ret), arglist)
    return structs, protos


def canon_c(t):
    t = " ".join(t.replace("const", " ").split())
    t = t.replace(" *", "*").replace("* ", "*")
    base = t.rstrip("*")
    stars = len(t) - len(base)
    base = {"int": "int32_t", "unsigned": "uint32_t"}.get(base.strip(), base.strip())
    return base + "*" * stars


def julia_to_c(t):
    """Canonical C type of a Julia ccall / field type."""
    t = t.strip()
    if t in SCALAR:
        return SCALAR[t]
    if t == "Cstring":
        return "char*"
    m = re.fullmatch(r"(Ptr|Ref)\{(.*)\}", t)
    if m:
        inner = m.group(2).strip()
        if inner in STRUCT_MAP:
            return STRUCT_MAP[inner] + "*"
        return julia_to_c(inner) + "*"
    raise AssertionError(f"unmapped Julia type {t!r}")


def compatible(jc, cc):
    """Julia-side canonical type vs C canonical type: Ptr{Cvoid} binds any pointer (opaque
    handles: mrbo_plan_t*, void* streams)."""
    if jc == cc:
        return True
    if jc.startswith("void*") and cc.endswith("*") and jc.count("*") <= cc.count("*"):
        return jc.count("*") == cc.count("*") or (jc == "void**" and cc.endswith("**"))
    return False


def julia_structs(src):
    out = {}
    for name, body in re.findall(rf"(?m)^struct\s+({IDENT})\s*\n(.*?)^end", src, flags=re.S):
        fields = re.findall(rf"(?m)^\s*({IDENT})::(\S+)", body)
        out[name] = fields
    return out


def julia_ccalls(src):
    calls = []
    for m in re.finditer(r"\bccall\s*\(", src):
        parts = split_top(call_body(src, m.end() - 1))
        fn = re.match(r"\(\s*:(\w+)\s*,", parts[0]).group(1)
        tup = parts[2].strip()
        assert tup.startswith("(") and tup.endswith(")"), tup
        types = split_top(tup[1:-1])
        calls.append((fn, parts[1].strip(), types, parts[3:]))
    return calls


@pytest.fixture(scope="module")
def shim():
    return strip_julia(open(SHIM, encoding="utf-8").read())


# ---------------------------------------------------------------------------------------------
def test_struct_mirrors_match_c_structs(shim):
    cstructs, _ = c_header()
    js = julia_structs(shim)
    for jname, cname in STRUCT_MAP.items():
        jf, cf = js[jname], cstructs[cname]
        assert [f for f, _ in jf] == [f for f, _ in cf] or len(jf) == len(cf), (jname, jf, cf)
        assert len(jf) == len(cf), f"{jname}: {len(jf)} fields, {cname}: {len(cf)}"
        for (jn, jt), (cn, ct) in zip(jf, cf):
            assert compatible(julia_to_c(jt), ct), f"{jname}.{jn}::{jt} vs {cname}.{cn} ({ct})"


def _offsets(fields):
    """C layout of a field list (canonical C types): natural alignment, as Julia isbits structs."""
    off, out, maxal = 0, [], 1
    for _, t in fields:
        k = "ptr" if t.endswith("*") else t
        sz = SIZE_ALIGN[k]
        off = (off + sz - 1) // sz * sz
        out.append(off)
        off += sz
        maxal = max(maxal, sz)
    return out, (off + maxal - 1) // maxal * maxal


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc needed for the C offsets")
def test_struct_offsets_match_compiled_header(shim):
    js = julia_structs(shim)
    cstructs, _ = c_header()
    prog = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, fields in cstructs.items():
        if cname not in STRUCT_MAP.values():
            continue
        for f, _ in fields:
            prog.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
        prog.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
    prog.append("return 0;}")
    with tempfile.TemporaryDirectory() as tmp:
        c = os.path.join(tmp, "off.c")
        open(c, "w").write("\n".join(prog))
        exe = os.path.join(tmp, "off")
        subprocess.check_call(["gcc", "-o", exe, c])
        lines = subprocess.check_output([exe], text=True).split("\n")
    got = {}
    for ln in lines:
        if ln:
            s, f, v = ln.split()
            got[(s, f)] = int(v)
    for jname, cname in STRUCT_MAP.items():
        jf = [(n, julia_to_c(t)) for n, t in js[jname]]
        offs, size = _offsets(jf)
        for (n, _), (cn, _), o in zip(jf, cstructs[cname], offs):
            assert got[(cname, cn)] == o, f"{jname}.{n} at {o}, C {cname}.{cn} at {got[(cname, cn)]}"
        assert got[(cname, "sizeof")] == size


def test_ccalls_match_prototypes(shim):
    _, protos = c_header()
    calls = julia_ccalls(shim)
    assert {c[0] for c in calls} >= {"mrbo_plan_create", "mrbo_plan_destroy", "mrbo_simulate_mc",
                                     "mrbo_simulate_ghq", "mrbo_base_solve", "mrbo_gp_fit", "mrbo_last_error"}
    for fn, ret, types, args in calls:
        assert fn in protos, f"ccall of {fn}, which include/mrbo.h does not declare"
        cret, cargs = protos[fn]
        assert compatible(julia_to_c(ret), cret) or (ret == "Cstring" and cret == "char*"), (fn, ret, cret)
        assert len(types) == len(cargs), f"{fn}: {len(types)} ccall types, C prototype has {len(cargs)}"
        for k, (jt, ct) in enumerate(zip(types, cargs)):
            assert compatible(julia_to_c(jt), ct), f"{fn} argument {k + 1}: {jt} vs {ct}"
        assert len(args) == len(types), f"{fn}: {len(args)} arguments passed for {len(types)} types"


def test_struct_constructor_calls_pass_every_field(shim):
    js = julia_structs(shim)
    n = 0
    for jname in STRUCT_MAP:
        for m in re.finditer(rf"\b{jname}\s*\(", shim):
            pre = shim[max(0, m.start() - 8):m.start()]
            if "struct" in pre or "Ref{" in shim[max(0, m.start() - 4):m.start()]:
                continue
            args = split_top(call_body(shim, m.end() - 1))
            assert len(args) == len(js[jname]), f"{jname}(…) with {len(args)} values for {len(js[jname])} fields"
            n += 1
    assert n >= 4


def _imports(shim):
    used, imported = set(), set()
    for kind, body in re.findall(r"(?m)^(using|import)\s+Main\s*:\s*((?:[^\n]*,\s*\n)*[^\n]*)", shim):
        names = {x.strip() for x in body.replace("\n", " ").split(",") if x.strip()}
        (imported if kind == "import" else used).update(names)
    return used, imported


def _locals(shim):
    loc = set()
    loc.update(re.findall(rf"({IDENT})\s*::", shim))                    # typed parameters / fields
    loc.update(re.findall(rf"(?<![.\w])({IDENT})\s*=(?!=)", shim))     # assignments and keyword params
    for grp in re.findall(r"\bfor\s+\(?([^=\n]*?)\)?\s+in\b", shim):
        loc.update(x.strip() for x in grp.split(","))
    for grp in re.findall(rf"(?m)^\s*((?:{IDENT}\s*,\s*)+{IDENT})\s*=", shim):
        loc.update(x.strip() for x in grp.split(","))
    loc.update(re.findall(rf"({IDENT})\s*->", shim))                    # lambda parameters
    loc.update(re.findall(rf"\(({IDENT})\s*->", shim))
    return loc


def test_reference_names_are_in_scope(shim):
    ref = json.load(open(NAMES, encoding="utf-8"))
    refnames = set(ref["names"])
    used, imported = _imports(shim)
    body = re.sub(r"(?m)^(using|import)\s+Main\s*:\s*((?:[^\n]*,\s*\n)*[^\n]*)", "", shim)
    defined = set(re.findall(rf"(?m)^(?:function|struct|mutable struct|const)\s+({IDENT})", body))
    defined |= set(re.findall(rf"(?m)^({IDENT})\s*\([^=\n]*\)\s*=", body))
    # identifiers not preceded by '.' (field access / qualified names)
    tokens = set(re.findall(rf"(?<![.\w])({IDENT})", body))
    local = _locals(body) - defined
    needed = sorted((tokens & refnames) - local - defined)
    missing = [n for n in needed if n not in used | imported]
    assert not missing, f"reference names used by MRBO.jl but not brought into scope from Main: {missing}"
    # the generic functions it adds methods to: reference names defined here must be imported
    extended = sorted(defined & refnames)
    assert "simulate_trajectory_mc" in extended and "simulate_trajectory_ghq" in extended
    assert set(extended) <= imported, f"methods of reference functions without `import Main:`: " \
                                      f"{sorted(set(extended) - imported)}"
    # and nothing is imported that the reference does not define (a typo would fail at load)
    assert (used | imported) <= refnames, sorted((used | imported) - refnames)
    # qualified package names must be bound in the module
    for pkg in set(re.findall(r"(?<![.\w])([A-Z]\w*)\.\w", body)):
        if pkg in ref["packages"]:
            assert re.search(rf"(?m)^(import|using)\s+{pkg}\b", shim), f"{pkg}. used without import {pkg}"


def test_exports_exist(shim):
    exp = set()
    for body in re.findall(r"(?m)^export\s+([^\n]*)", shim):
        exp.update(x.strip() for x in body.split(","))
    defined = set(re.findall(rf"(?m)^(?:function|struct|mutable struct|const)\s+({IDENT})", shim))
    defined |= set(re.findall(rf"(?m)^({IDENT})\s*\(", shim))
    assert exp and exp <= defined, sorted(exp - defined)
    assert "MrboBackend" in exp


def test_integration_doc_matches_the_shim():
    doc = open(os.path.join(ROOT, "INTEGRATION.md"), encoding="utf-8").read()
    src = open(SHIM, encoding="utf-8").read()
    assert "using .MRBO" in doc and re.search(r"(?m)^module MRBO\b", src)
    for name in re.findall(r"\b(mrbo_\w+!?)\(", doc):
        if name.endswith("!") or name in ("mrbo_log_likelihood",):
            assert re.search(rf"(?m)^function {re.escape(name)}\(", src), name


def _functions(shim):
    """(name, body) of every top-level `function … end` block (the shim indents bodies, so a
    function ends at the first `end` in column 0)."""
    return re.findall(rf"(?ms)^function\s+({IDENT})\s*\((.*?)^end\b", shim)


def test_plan_lifecycle_is_deterministic(shim):
    """Every device plan the shim creates is released deterministically: no
    GC finalizer (Julia's GC does not see device memory); a function that calls mrbo_plan_create
    directly destroys the handle in a `finally` block unless it is the MrboPlan constructor; every
    MrboPlan(…) construction outside the constructor goes into the bounded plan cache; the cache's
    eviction and release path calls mrbo_plan_destroy!, which calls mrbo_plan_destroy; and the
    rollout methods (R = 1, batched, Gauss–Hermite) take their plans from that cache."""
    assert "finalizer(" not in shim
    funcs = _functions(shim)
    names = [n for n, _ in funcs]
    body = dict(zip(names, (b for _, b in funcs)))
    creators = [n for n, b in funcs if "mrbo_plan_create" in b]
    assert creators, "no mrbo_plan_create call found"
    for n, b in funcs:
        if "mrbo_plan_create" not in b or n == "MrboPlan":
            continue
        fin = b.split("finally", 1)
        assert len(fin) == 2 and "mrbo_plan_destroy" in fin[1], f"{n}: plan created without try … finally destroy"
    # constructions of MrboPlan(…) with surrogate arguments outside the constructor itself
    for n, b in funcs:
        if n == "MrboPlan":
            continue
        for m in re.finditer(r"\bMrboPlan\s*\(", b):
            assert n == "mrbo_cached_plan", f"{n} builds an MrboPlan outside the cache"
    cp = body["mrbo_cached_plan"]
    assert "PLAN_CACHE[key] = p" in cp and "MRBO_PLAN_CACHE_MAX" in cp and "mrbo_release_plans!()" in cp
    assert "mrbo_plan_destroy!(p)" in body["mrbo_release_plans!"] and "empty!(PLAN_CACHE)" in body["mrbo_release_plans!"]
    assert "mrbo_plan_destroy" in body["mrbo_plan_destroy!"] and "C_NULL" in body["mrbo_plan_destroy!"]
    assert "atexit(mrbo_release_plans!)" in body["__init__"]
    uses = [b for n, b in funcs if n in ("simulate_trajectory_mc", "simulate_trajectory_ghq")]
    # two simulate_trajectory_mc methods (R = 1 and batched) + the ghq method
    assert len(uses) == 3 and all("mrbo_cached_plan(" in b for b in uses)


def test_batched_method_shapes(shim):
    """The batched simulate_trajectory_mc method (one launch for the x0 batch of generate_batch,
    utils.jl:97-106) passes R = size(X0, 2) to its plan and M×R / d×M×R containers to the C ABI,
    and returns one ExpectedTrajectoryOutput per restart."""
    funcs = [b for n, b in _functions(shim) if n == "simulate_trajectory_mc"]
    bat = [b for b in funcs if "X0::Matrix{Float64}" in b]
    assert len(bat) == 1
    b = bat[0]
    assert "R = R" in b and "d, R = size(X0)" in b and "zeros(Int32, M, R)" in b
    assert "for r in 1:R]" in b and "mrbo_eto(" in b
