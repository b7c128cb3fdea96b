"""Parse include/spai_hip.h into ctypes signatures (test helper, no GPU).

Every entry point of the C ABI is declared as ``<ret> spai_name(<params>);``.  Each parameter's C
type maps to the ctypes type a binding must pass: pointers -> c_void_p (``const char*`` ->
c_char_p), fixed-width integers to their ctypes twins, ``size_t`` -> c_size_t.  Used to check the
package's own binding (``_lib.SIGNATURES``) and the reference-side stub published in
INTEGRATION.md against the header, argument for argument.
"""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "spai_hip.h")
INTEGRATION = os.path.join(ROOT, "INTEGRATION.md")

_SCALARS = {
    "int": ctypes.c_int, "int32_t": ctypes.c_int32, "int64_t": ctypes.c_int64, "uint64_t": ctypes.c_uint64,
    "size_t": ctypes.c_size_t, "double": ctypes.c_double, "float": ctypes.c_float,
}


def ctype_of(decl: str):
    """ctypes type of one C parameter declaration (with or without its name) or return type."""
    d = " ".join(decl.replace("*", " * ").split())
    if d == "void":
        return None
    toks = d.split()
    if "*" in toks:
        base = [t for t in toks[:toks.index("*")] if t != "const"]
        return ctypes.c_char_p if base == ["char"] else ctypes.c_void_p
    toks = [t for t in toks if t != "const"]
    if toks[0] not in _SCALARS:
        raise ValueError(f"unknown C type in {decl!r}")
    return _SCALARS[toks[0]]


def parse_header(path: str = HEADER) -> dict:
    """{name: (restype, [argtypes], [parameter names])} of every spai_* declaration."""
    text = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
    text = re.sub(r"#[^\n]*", "", text)
    out = {}
    for ret, name, params in re.findall(r"([A-Za-z_][\w\s\*]*?)\b(spai_\w+)\s*\(([^)]*)\)\s*;", text):
        ret = ret.split()[-2:] if "const" in ret else ret.split()[-1:]
        restype = ctype_of(" ".join(ret))
        plist = [p.strip() for p in params.split(",") if p.strip()]
        if plist == ["void"]:
            plist = []
        names = [re.findall(r"\w+", p)[-1] for p in plist]
        out[name] = (restype, [ctype_of(p.rsplit(None, 1)[0] if not p.endswith("*") else p) for p in plist], names)
    return out


def integration_stub() -> str:
    """The Python code block under INTEGRATION.md's 'Reference-side binding' heading."""
    text = open(INTEGRATION).read()
    sec = text.split("### Reference-side binding", 1)[1]
    m = re.search(r"```python\n(.*?)```", sec, flags=re.S)
    return m.group(1)
