"""The Java FFM binding (java/net/bowen/system/RtAmd.java) against the C ABI.

There is no JDK in this image, so the Java sources cannot be compiled here; this
CPU test checks what can be checked without one: every rt_* function the binding
looks up is declared in include/rt/rt.h and exported by librtamd.so, and each
downcall's FunctionDescriptor has the C prototype's return kind and parameter
kinds in order (int -> JAVA_INT, float -> JAVA_FLOAT, size_t / uint64_t ->
JAVA_LONG, pointers -> ADDRESS).  The executor mirror (RtAmdRaytraceExecutor.java)
keeps the reference RaytraceExecutor's public methods (RaytraceExecutor.java:16-157).
"""
import os
import re

import rtamd

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(REPO, "java", "net", "bowen", "system")
HEADER = os.path.join(REPO, "include", "rt", "rt.h")


def _c_prototypes():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    protos = {}
    for m in re.finditer(r"^\s*([A-Za-z_][\w\s\*]*?)\s*\*?\s*(rt_\w+)\s*\(([^)]*)\)\s*;", text, flags=re.M):
        ret = m.group(0).split(m.group(2))[0].strip()
        args = [a.strip() for a in m.group(3).split(",") if a.strip() and a.strip() != "void"]
        protos[m.group(2)] = (ret, args)
    return protos


def _kind(ctype):
    c = ctype.replace("const", "").strip()
    if "*" in c or "[" in c:
        return "ADDRESS"
    base = c.split()[0]
    return {"int": "JAVA_INT", "float": "JAVA_FLOAT", "size_t": "JAVA_LONG", "uint64_t": "JAVA_LONG"}[base]


def _java_downcalls():
    src = open(os.path.join(JAVA, "RtAmd.java")).read()
    out = {}
    for m in re.finditer(r'fn\("(rt_\w+)",\s*FunctionDescriptor\.of\(([^)]*)\)\)', src):
        kinds = [k.strip() for k in m.group(2).split(",")]
        out[m.group(1)] = (kinds[0], kinds[1:])
    return out


def test_binding_matches_header_and_library():
    protos = _c_prototypes()
    calls = _java_downcalls()
    assert len(calls) >= 13, sorted(calls)
    lib = rtamd.amd()
    for name, (ret, params) in calls.items():
        assert name in protos, f"{name} is not declared in rt.h"
        assert hasattr(lib, name), f"{name} is not exported by librtamd.so"
        c_ret, c_args = protos[name]
        assert ret == _kind(c_ret), (name, ret, c_ret)
        assert params == [_kind(a.rsplit(" ", 1)[0] if not a.endswith("]") else a) for a in c_args], (name, params, c_args)


def test_executor_mirror_keeps_the_reference_methods():
    src = open(os.path.join(JAVA, "RtAmdRaytraceExecutor.java")).read()
    for sig in ["void setSamplePerPixel(int", "void resetCompleteState()", "int getNumSamples()",
                "int getSamplePerPixel()", "int getFinishTime()", "String getFinishTimeString()",
                "int getLastDispatchTime()", "void addCompleteListener(Runnable", "void raytrace()",
                "boolean sampleComplete()"]:
        assert f"public {sig}" in src, sig
