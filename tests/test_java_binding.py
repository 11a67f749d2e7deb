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


PATCH = os.path.join(REPO, "java", "patches", "rtamd-dropin.patch")


def _patch_files():
    files, cur = {}, None
    for line in open(PATCH):
        if line.startswith("+++ "):
            cur = line.split()[1].split("/src/main/java/", 1)[1]
            files[cur] = {"+": [], "-": []}
        elif cur and line[:1] in "+-" and not line.startswith(("+++", "---")):
            files[cur][line[0]].append(line[1:].rstrip("\n"))
    return files


def test_dropin_patch_replaces_every_gl_call_site():
    """java/patches/rtamd-dropin.patch (against the reference tree) switches each hot-path
    GL call site of SURVEY §8b to the C ABI: the six SSBO uploads of RaytraceModel.put*ToProgram
    (RaytraceModel.java:115-246), Texture.putData's glTexImage2D and putTextureIndices
    (Texture.java:122-133, 238-247), Camera.putToShaderProgram's UBO + background uniform
    (Camera.java:121-143), Window.initRaytraceExecutor / saveImage / resize / loop
    (Window.java:116-129, 213-238, 250-281) and GuiRenderer.maxDepthUpdate (GuiRenderer.java:64-68)."""
    f = _patch_files()
    rm = f["net/bowen/draw/models/raytrace/RaytraceModel.java"]
    for ssbo, binding in [("sphereSSBO", "SPHERES"), ("quadSSBO", "QUADS"), ("boxesSSBO", "BOXES"),
                          ("constantMediumSSBO", "MEDIA"), ("bvhSSBO", "BVH"), ("lightsSSBO", "LIGHTS")]:
        assert any(f"{ssbo}.uploadData(buffer, GL_STATIC_DRAW);" in l for l in rm["-"]), ssbo
        assert any(f"RtAmdBackend.upload(RtAmd.{binding}, buffer);" in l for l in rm["+"]), binding
    tx = f["net/bowen/draw/textures/Texture.java"]
    assert sum("RtAmdBackend.putTexture(this, internalFormat, format, type, width, height, data);" in l
               for l in tx["+"]) == 2
    assert any("RtAmdBackend.uploadTextures(TEXTURES_IN_COMPUTE);" in l for l in tx["+"])
    cam = f["net/bowen/draw/models/raytrace/Camera.java"]
    assert any("ubo.uploadData(buffer, GL_STATIC_DRAW);" in l for l in cam["-"])
    assert any('setUniform3fv("background"' in l for l in cam["-"])
    assert any("RtAmdBackend.setCamera(buffer, background.asArray());" in l for l in cam["+"])
    win = f["net/bowen/gui/Window.java"]
    assert any("new RaytraceExecutor(screenQuadTexture, computeProgram)" in l for l in win["-"])
    assert any("new RtAmdRaytraceExecutor(RtAmdBackend.get())" in l for l in win["+"])
    assert any("screenQuadTexture.saveAsPNG(outputFile);" in l for l in win["-"])
    assert any("RtAmdBackend.saveAsPNG(outputFile)" in l for l in win["+"])
    assert any("RtAmdBackend.get().resize(width, height);" in l for l in win["+"])
    gui = f["net/bowen/gui/GuiRenderer.java"]
    assert any('setUniform1iv("max_depth"' in l for l in gui["-"])
    assert any("raytraceExecutor.setMaxDepth(maxDepth[0]);" in l for l in gui["+"])


def _methods(java_file):
    src = open(os.path.join(JAVA, java_file)).read()
    return set(re.findall(r"public (?:static )?(?:synchronized )?[\w\[\]<>]+ (\w+)\(", src)), src


def test_dropin_calls_resolve_to_the_binding():
    """Every RtAmdBackend / RtAmd / executor method the patched call sites and the backend use exists."""
    backend, bsrc = _methods("RtAmdBackend.java")
    rt, _ = _methods("RtAmd.java")
    ex, _ = _methods("RtAmdRaytraceExecutor.java")
    used = set()
    for fl in _patch_files().values():
        for line in fl["+"]:
            used |= {("B", m) for m in re.findall(r"RtAmdBackend\.(\w+)\(", line)}
            used |= {("E", m) for m in re.findall(r"raytraceExecutor\.(\w+)\(", line)}
    for kind, m in sorted(used):
        assert m in (backend if kind == "B" else ex), (kind, m)
    for m in set(re.findall(r"(?:get\(\)|\br)\.(\w+)\(", bsrc)):
        assert m in rt, m


def test_binding_allocates_per_call():
    """RtAmd keeps no long-lived arena: every call's native arguments come from a confined arena
    closed when the call returns (the context arena grew by 33 MB per readImage)."""
    src = open(os.path.join(JAVA, "RtAmd.java")).read()
    assert "private final Arena" not in src and "arena." not in src
    n_alloc = len(re.findall(r"\ba\.allocate", src))
    n_scopes = len(re.findall(r"try \(Arena a = Arena\.ofConfined\(\)\)", src))
    assert n_alloc >= 10 and n_scopes >= 10


def test_executor_polls_dispatch_time_without_waiting():
    """getLastDispatchTime refreshes on every raytrace() from the previous render's device time
    when it is ready (rt_render_done), as the reference polls its finished timer queries."""
    src = open(os.path.join(JAVA, "RtAmdRaytraceExecutor.java")).read()
    body = _java_method(src, "private int launch(int n)")
    assert "rt.renderDoneNanos()" in body and "lastDispatchTime" in body


def _java_method(src, signature):
    body = src[src.index(signature):]
    return body[:body.index("\n    }\n")]


def _clamp_frames_py(src):
    """RtAmdRaytraceExecutor.clampFrames translated statement by statement into Python (its
    body is two Java statements over ints: an if with Math.min, then a return of Math.max)."""
    body = _java_method(src, "static int clampFrames(int n, int numSamples, int samplePerPixel)")
    stmts = [s.strip() for s in body.split("{", 1)[1].split(";") if s.strip()]
    assert len(stmts) == 2, stmts
    m = re.fullmatch(r"if \((\w+ > 0)\) n = Math\.min\((.+)\)", stmts[0])
    assert m, stmts[0]
    r = re.fullmatch(r"return Math\.max\((.+)\)", stmts[1])
    assert r, stmts[1]
    py = (f"def clamp(n, numSamples, samplePerPixel):\n"
          f"    if {m.group(1)}: n = min({m.group(2)})\n"
          f"    return max({r.group(1)})\n")
    ns = {}
    exec(py, ns)
    return ns["clamp"]


def test_dropin_renders_exactly_sample_per_pixel():
    """the patched Window loop calls raytrace(FRAMES_PER_DISPLAY) while
    !sampleComplete(); the reference renders exactly samplePerPixel frames (RaytraceExecutor.java:
    100-156, Window.java:250-281; CLI default 20, Main.java:36).  raytrace(int) clamps to the
    frames still missing, so with spp 20 and 16 frames per display the launches are 16 then 4."""
    src = open(os.path.join(JAVA, "RtAmdRaytraceExecutor.java")).read()
    pub = _java_method(src, "public int raytrace(int n)")
    assert "launch(clampFrames(n, numSamples, samplePerPixel))" in pub
    assert "launch(1)" in _java_method(src, "public void raytrace()")   # unclamped, as the reference
    clamp = _clamp_frames_py(src)
    win = _patch_files()["net/bowen/gui/Window.java"]["+"]
    per_display = int(re.search(r'getInteger\("rtamd.framesPerDisplay", (\d+)\)', "\n".join(win)).group(1))
    assert any("if (!raytraceExecutor.sampleComplete())" in l for l in win)
    assert any("raytraceExecutor.raytrace(FRAMES_PER_DISPLAY);" in l for l in win)

    def loop(spp, per):
        num, calls = 0, []
        while not num >= spp:               # sampleComplete(): numSamples >= samplePerPixel
            k = clamp(per, num, spp)
            assert k > 0
            calls.append(k)
            num += k
        return calls, num

    assert per_display == 16
    assert loop(20, per_display) == ([16, 4], 20)
    for spp in (1, 15, 16, 17, 32, 33, 4096):
        for per in (1, 7, 16, 64):
            calls, num = loop(spp, per)
            assert num == spp and all(c <= per for c in calls), (spp, per, calls)
    assert clamp(16, 20, 20) == 0 and clamp(16, 25, 20) == 0      # nothing past spp
    assert clamp(16, 100, 0) == 16 and clamp(-3, 0, 20) == 0       # unbounded; non-positive n
