"""CPU: the C-ABI library loads and exports every entry point include/gelly_hip.h declares.
No compute call is made here (no GPU in the build container)."""
import ctypes
import re
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "gelly_hip.h"


def declared():
    return sorted(set(re.findall(r"^GS_API\s+[\w\s\*]+?\b(gs_\w+)\s*\(", HEADER.read_text(), re.M)))


def test_header_declares_abi():
    names = declared()
    assert "gs_window_reduce" in names and "gs_window_triangles" in names and len(names) >= 18


def test_library_exports_every_declared_symbol(pkg):
    lib = pkg.load_library()
    so = Path(lib._name)
    out = subprocess.run(["nm", "-D", "--defined-only", str(so)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gs_\w+)", out))
    missing = [n for n in declared() if n not in exported]
    assert not missing, f"declared but not exported: {missing}"
    for n in declared():
        assert getattr(lib, n) is not None
    from gelly_streaming_amd import _lib
    assert sorted(_lib.EXPORTS) == declared()


def test_abi_version_and_no_device_error(pkg):
    lib = pkg.load_library()
    want = int(re.search(r"#define GS_ABI_VERSION (\d+)", HEADER.read_text()).group(1))
    assert want == 2 and lib.gs_abi_version() == want
    java = re.search(r"GS_ABI_VERSION = (\d+);", GELLYHIP_JAVA.read_text()).group(1)
    assert int(java) == want   # the JNI binding refuses a library of another ABI
    import torch
    if not torch.cuda.is_available():
        # lifecycle only: gs_create must fail cleanly (status, no abort) when no HIP device exists
        ctx = ctypes.c_void_p()
        from gelly_streaming_amd import _lib
        st = lib.gs_create(ctypes.byref(_lib.GsConfig(0, 0, 0)), ctypes.byref(ctx))
        assert st == _lib.GS_EDEVICE and not ctx.value
        assert lib.gs_last_error(None) == b"null context"


def test_engine_fails_loudly_without_device(pkg):
    import pytest
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pkg.GsError):
        pkg.Engine(0)


STRUCTS = {"gs_config": "GsConfig", "gs_edge_batch": "GsEdgeBatch", "gs_vertex_out": "GsVertexOut",
           "gs_degree_out": "GsDegreeOut", "gs_csr_out": "GsCsrOut", "gs_pair_out": "GsPairOut",
           "gs_pair_batch": "GsPairBatch", "gs_stage_times": "GsStageTimes", "gs_partials_out": "GsPartialsOut",
           "gs_partial_batch": "GsPartialBatch", "gs_stream_config": "GsStreamConfig",
           "gs_window_result": "GsWindowResult", "gs_stream_stats_t": "GsStreamStats"}


def test_struct_layouts_match_header(pkg):
    """ctypes mirrors of the ABI structs have the sizes and field offsets the C compiler gives them."""
    from gelly_streaming_amd import _lib
    lines, want = [], []
    for c_name, py_name in STRUCTS.items():
        t = getattr(_lib, py_name)
        lines.append(f'printf("%zu\\n", sizeof({c_name}));')
        want.append(ctypes.sizeof(t))
        for f, _ in t._fields_:
            lines.append(f'printf("%zu\\n", offsetof({c_name}, {f}));')
            want.append(getattr(t, f).offset)
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"gelly_hip.h\"\nint main(){" + "".join(lines) + "}"
    tmp = ROOT / "gpurun_out"
    tmp.mkdir(exist_ok=True)
    (tmp / "sz.c").write_text(src)
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(tmp / "sz.c"), "-o", str(tmp / "sz")], check=True)
    got = [int(x) for x in subprocess.run([str(tmp / "sz")], capture_output=True, text=True).stdout.split()]
    assert got == want


# ---- the Java side (java/): JNI binding, shim and dispatch patch (source-only: no JDK in this image) ----
JAVA = ROOT / "java"
GELLYHIP_JAVA = JAVA / "src/main/java/org/apache/flink/graph/streaming/gpu/GellyHip.java"
SHIM = JAVA / "src/main/c/gellyhip_jni.c"


def test_java_constants_match_header():
    """Every GS_* constant GellyHip.java defines has the header's value (enum ordinals, status codes,
    stream kinds), as the C compiler sees the header."""
    consts = dict(re.findall(r"public static final int (GS_\w+) = (-?\d+);", GELLYHIP_JAVA.read_text()))
    assert len(consts) >= 30 and consts["GS_DIR_OUT"] == "1"
    names = sorted(consts)
    src = ("#include <stdio.h>\n#include \"gelly_hip.h\"\nint main(){" +
           "".join(f'printf("%lld\\n", (long long)({n}));' for n in names) + "}")
    tmp = ROOT / "gpurun_out"
    tmp.mkdir(exist_ok=True)
    (tmp / "jconst.c").write_text(src)
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(tmp / "jconst.c"), "-o", str(tmp / "jconst")], check=True)
    got = subprocess.run([str(tmp / "jconst")], capture_output=True, text=True, check=True).stdout.split()
    assert dict(zip(names, got)) == {n: consts[n] for n in names}


def test_jni_shim_covers_every_native_and_calls_only_declared_entry_points():
    natives = set(re.findall(r"static native [\w\[\]]+ (\w+)\(", GELLYHIP_JAVA.read_text()))
    shim = SHIM.read_text()
    implemented = set(re.findall(r"JNI_FN\((\w+)\)", shim)) - {"name"}   # the macro definition itself
    assert natives and natives == implemented, (natives ^ implemented)
    called = set(re.findall(r"\b(gs_\w+)\(", shim))
    assert called <= set(declared()), called - set(declared())


def test_dispatch_patch_applies_to_the_reference():
    """java/patches/*.patch (GraphWindowStream's package-private ctor + built-in dispatch, slice() passing
    the pre-keyBy edges) applies cleanly to the reference tree (checked without writing to it)."""
    import pytest
    ref = Path("/root/reference")
    if not (ref / "src").is_dir():
        pytest.skip("reference tree not present (GPU box)")
    for patch in sorted((JAVA / "patches").glob("*.patch")):
        r = subprocess.run(["git", "apply", "--check", str(patch)], cwd=ref, capture_output=True,
                           text=True)
        assert r.returncode == 0, r.stderr


GPU_JAVA = JAVA / "src/main/java/org/apache/flink/graph/streaming/gpu"
PATCH = JAVA / "patches/gelly-streaming-gpu-dispatch.patch"


def test_every_builtin_marker_reaches_a_native_and_an_entry_point():
    """SURVEY.md §8(b) dispatch rule, end to end on the Java side: every built-in marker (GpuBuiltins'
    reducers and folds, and the reference's GenerateCandidateEdges, which the patch marks BuiltinApply)
    is dispatched by the patch to an operator; WindowTriangles.main is routed to the TRIANGLES stream;
    every GellyHip native an operator calls is declared, implemented by the JNI shim, and the shim calls
    only entry points include/gelly_hip.h declares."""
    builtins = (GPU_JAVA / "GpuBuiltins.java").read_text()
    markers = {m.group(1): m.group(2) for m in re.finditer(
        r"public static final class (\w+)(?:<[^>]*>)?\s+implements[^{]*?\b(Builtin(?:Fold|Apply)?)\b", builtins)}
    assert {"SumReduce", "MinReduce", "MaxReduce", "CountFold", "SumValuesFold", "DegreeMaxNeighborFold"} <= set(markers)
    patch = PATCH.read_text()
    added = "\n".join(line[1:] for line in patch.splitlines() if line.startswith("+") and not line.startswith("+++"))
    after = "\n".join(line[1:] for line in patch.splitlines() if line[:1] in (" ", "+") and not line.startswith("+++"))
    assert re.search(r"GenerateCandidateEdges implements\s*EdgesApply<[^{]*GpuBuiltins\.BuiltinApply \{", after)
    markers["GenerateCandidateEdges"] = "BuiltinApply"
    # marker interface -> (dispatch test in the patch, the operator it builds, the stream kind it asks for)
    # (marker -> dispatch test, the operator factory the patch calls, the stream kind it asks for); each
    # factory builds its operator
    route = {"Builtin": ("GpuBuiltins.Builtin", "GpuWindowOperator.neighborhood(", "GS_STREAM_REDUCE"),
             "BuiltinFold": ("GpuBuiltins.BuiltinFold", "GpuWindowOperator.neighborhood(", "GS_STREAM_FOLD"),
             "BuiltinApply": ("GpuBuiltins.BuiltinApply", "GpuCandidatesOperator.applyOnNeighbors(", None)}
    for name, iface in markers.items():
        test, factory, kind = route[iface]
        assert f"instanceof {test}" in added, (name, test)
        assert factory in added, (name, factory)
        cls = factory.split(".")[0]
        assert f"new {cls}" in (GPU_JAVA / f"{cls}.java").read_text(), (name, cls)
        if kind:
            assert kind in added, (name, kind)
    # ConnectedComponents: SimpleEdgeStream.aggregate routes it to GpuComponentsOperator
    assert "instanceof ConnectedComponents" in added and "GpuComponentsOperator.connectedComponents(" in added
    assert "getWindowMillis()" in added
    assert "GS_STREAM_DEGREE_MAX" in added
    # WindowTriangles.main: slice -> candidates -> CountTriangles -> timeWindowAll.sum on one operator
    assert "GpuWindowOperator.windowTriangles(" in added
    assert "GS_STREAM_TRIANGLES" in (GPU_JAVA / "GpuWindowOperator.java").read_text()
    natives = set(re.findall(r"static native [\w\[\]]+ (\w+)\(", GELLYHIP_JAVA.read_text()))
    bodies = {re.search(r"JNI_FN\((\w+)\)", chunk).group(1): chunk
              for chunk in SHIM.read_text().split("JNIEXPORT")[1:]}
    for op in ("GpuWindowOperator", "GpuCandidatesOperator", "GpuComponentsOperator"):
        used = set(re.findall(r"GellyHip\.([a-z]\w*)\(", (GPU_JAVA / f"{op}.java").read_text())) - {"direct"}
        assert used and used <= natives, (op, used - natives)
        for n in used:
            calls = set(re.findall(r"\b(gs_\w+)\(", bodies[n]))
            assert calls and calls <= set(declared()), (op, n, calls)


def test_dispatch_falls_back_for_unsupported_types():
    """A built-in over edges the engine does not take (non-Long keys, values that are not Integer / Long /
    Float / Double) stays on Flink: the patch's gpu() asks GpuBuiltins.supports before dispatching."""
    patch = PATCH.read_text()
    assert "GpuBuiltins.supports(" in patch
    src = (GPU_JAVA / "GpuBuiltins.java").read_text()
    body = re.search(r"public static boolean supports\([^)]*\) \{([\s\S]*?)\n\t\}", src).group(1)
    assert "keyClass != Long.class" in body and "dtypeOf(valueClass)" in body


def _header_arity():
    """entry point -> number of parameters, from include/gelly_hip.h"""
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    out = {}
    for m in re.finditer(r"GS_API\s+[\w\s\*]+?\b(gs_\w+)\s*\(([^)]*)\)\s*;", text):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_panama_binding_matches_header():
    """java/.../GellyHipPanama.java (JDK 22 FFM, north_star's "Panama FFI"): every entry point it looks up
    is declared in gelly_hip.h with as many parameters as its FunctionDescriptor has arguments, and its
    struct layouts have the header's field offsets (as the C compiler lays them out)."""
    src = (GPU_JAVA / "GellyHipPanama.java").read_text()
    arity = _header_arity()
    found = re.findall(r'fn\("(gs_\w+)",\s*FunctionDescriptor\.(of|ofVoid)\(([^;]*?)\)\);', src)
    assert len(found) >= 8
    for name, kind, args in found:
        n = len([a for a in args.split(",") if a.strip()]) - (1 if kind == "of" else 0)
        assert name in arity and arity[name] == n, (name, n, arity.get(name))
    # struct layouts: field order / widths against offsetof() from the C compiler
    layouts = {"CONFIG": "gs_config", "EDGE_BATCH": "gs_edge_batch", "VERTEX_OUT": "gs_vertex_out",
               "DEGREE_OUT": "gs_degree_out", "PAIR_OUT": "gs_pair_out"}
    size = {"JAVA_INT": 4, "JAVA_LONG": 8, "ADDRESS": 8}
    prog = ["#include <stdio.h>", "#include <stddef.h>", '#include "gelly_hip.h"', "int main(){"]
    want = []
    for jl, cs in layouts.items():
        body = re.search(jl + r" = MemoryLayout\.structLayout\(([^;]*)\);", src).group(1)
        off = 0
        for ty, field in re.findall(r"(JAVA_INT|JAVA_LONG|ADDRESS)\.withName\(\"(\w+)\"\)", body):
            off = (off + size[ty] - 1) // size[ty] * size[ty]
            prog.append(f'printf("%zu\\n", offsetof({cs}, {field}));')
            want.append(off)
            off += size[ty]
    prog.append("}")
    tmp = ROOT / "gpurun_out"
    tmp.mkdir(exist_ok=True)
    (tmp / "panama_off.c").write_text("\n".join(prog))
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(tmp / "panama_off.c"), "-o", str(tmp / "panama_off")],
                   check=True)
    got = [int(x) for x in subprocess.run([str(tmp / "panama_off")], capture_output=True, text=True,
                                          check=True).stdout.split()]
    assert got == want


def _statements(text, token):
    """the Java statements (up to the next ';') that contain token"""
    out, at = [], 0
    while (i := text.find(token, at)) >= 0:
        start = text.rfind(";", 0, i) + 1
        start = max(start, text.rfind("{", 0, i) + 1, text.rfind("}", 0, i) + 1)
        end = text.find(";", i)
        out.append(text[start:end + 1])
        at = i + len(token)
    return out


def test_gpu_operators_keep_the_keyby_contract():
    """SURVEY.md §8(b) "Threading" / keyBy (SimpleEdgeStream.java:159-167): Flink runs an operator at the
    environment's parallelism (TestSlice's mini-cluster and the local env: several subtasks), and keyBy
    gives every record of a vertex to ONE subtask.  So every GPU operator the patch or the factories build
    is pinned: `transform(...)` is followed by `.setParallelism(1)`, or by `.setParallelism(p)` with a
    partitionCustom by the owner in the same statement; and no operator hard-codes a device (each
    subtask's gs_ctx goes to GpuBuiltins.deviceFor(subtask index))."""
    patch = PATCH.read_text()
    added = "\n".join(line[1:] for line in patch.splitlines() if line.startswith("+") and not line.startswith("+++"))
    sources = {"patch": added}
    for f in GPU_JAVA.glob("Gpu*Operator.java"):
        sources[f.name] = f.read_text()
    n = 0
    for where, text in sources.items():
        for st in _statements(text, ".transform("):
            n += 1
            m = re.search(r"\.setParallelism\((\w+)\)", st)
            assert m, (where, st)
            if m.group(1) != "1":
                assert "partitionCustom(" in st, (where, st)
        for st in _statements(text, "GellyHip.create("):
            assert "GpuBuiltins.deviceFor(" in st or re.search(r"create\(device,", st), (where, st)
            if "create(device," in st:   # the device variable comes from deviceFor in the same method
                assert re.search(r"final int device = GpuBuiltins\.deviceFor\(", text), where
    assert n >= 5
    # the owner routing is keyed the way the library filters (gs_candidates_begin_part)
    cand = (GPU_JAVA / "GpuCandidatesOperator.java").read_text()
    assert "RouteToOwners" in cand and "TargetPartitioner" in cand and "candidatesBegin(ctx, w.src, w.dst, w.n, parts, part)" in cand


def test_java_owner_function_is_the_librarys():
    """GpuBuiltins.ownerOf (the Flink partitioner) restates gs_owner_of (gs_ops.hpp owner_of): the same
    multipliers, shifts and multiply-high, so a vertex's records reach the subtask whose
    gs_candidates_begin_part emits it."""
    java = (GPU_JAVA / "GpuBuiltins.java").read_text()
    body = re.search(r"public static int ownerOf\(long v, int nparts\) \{([\s\S]*?)\n\t\}", java).group(1)
    cpp = (ROOT / "gelly-streaming_amd/csrc/gs_ops.hpp").read_text()
    cbody = re.search(r"owner_of\(int64_t v, uint32_t nparts\) \{([\s\S]*?)\n\}", cpp).group(1)
    jm = [int(x, 16) for x in re.findall(r"0x([0-9a-f]+)L", body)]
    cm = [int(x, 16) for x in re.findall(r"0x([0-9a-f]+)ull", cbody)]
    assert jm == cm and len(cm) == 2
    assert re.findall(r">>> (\d+)", body)[:3] == re.findall(r">> (\d+)", cbody)[:3] == ["33", "33", "33"]
    assert "((x >>> 32) * (long) nparts) >>> 32" in body and "((x >> 32) * (uint64_t)nparts) >> 32" in cbody


JNI_STUB = r"""
/* test infrastructure: the jni.h subset gellyhip_jni.c uses, so gcc can type-check the shim here
 * (no JDK in this image); the real header comes from the JDK at java/Makefile build time */
#include <stdint.h>
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_TRUE 1
#define JNI_FALSE 0
typedef int32_t jint; typedef int64_t jlong; typedef uint8_t jboolean; typedef jint jsize;
typedef void* jobject; typedef jobject jclass; typedef jobject jstring; typedef jobject jarray;
typedef jarray jlongArray; typedef jarray jobjectArray; typedef jint jthrowable;
struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
  void* (*GetDirectBufferAddress)(JNIEnv*, jobject);
  jobject (*NewDirectByteBuffer)(JNIEnv*, void*, jlong);
  jclass (*FindClass)(JNIEnv*, const char*);
  jint (*ThrowNew)(JNIEnv*, jclass, const char*);
  jlongArray (*NewLongArray)(JNIEnv*, jsize);
  void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
  void (*SetObjectArrayElement)(JNIEnv*, jobjectArray, jsize, jobject);
};
"""


def test_jni_shim_type_checks_against_the_header():
    """gcc -fsyntax-only of java/src/main/c/gellyhip_jni.c against include/gelly_hip.h (with a stub of
    the jni.h subset it uses): every ABI call in the shim has the header's argument types and count."""
    tmp = ROOT / "gpurun_out" / "jni_stub"
    tmp.mkdir(parents=True, exist_ok=True)
    (tmp / "jni.h").write_text(JNI_STUB)
    r = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Werror", "-Wno-unused-parameter", "-I", str(tmp), "-I",
                        str(ROOT / "include"), str(SHIM)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
