"""Build the native libraries in-tree (they travel to the GPU box with the repo).

  rpkt_amd/_build/librpkt_gpu.so   HIP engine for gfx950 + C ABI (include/rpkt_gpu.h);
                                   RCCL (rpkt_gpu_flow_reduce) is resolved at first use
  rpkt_amd/_build/librpkt_gen.so   host C++ synthetic frame generator

hipcc cross-compiles gfx950 without a GPU.  Rebuilds only when a source is newer.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(HERE, "_build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RPKT_OFFLOAD_ARCH", "gfx950")
ROCM_LIB = "/opt/rocm/lib"

GPU_LIB = os.path.join(OUT, "librpkt_gpu.so")
# the same units with -DRPKT_ABLATE: the product entry points plus the development hooks
# (kernel ablation variants, streaming references) that tools/ and bench.py's
# copy_ceiling call; the product library exports exactly include/rpkt_gpu.h
ABLATE_LIB = os.path.join(OUT, "librpkt_gpu_ablate.so")
GEN_LIB = os.path.join(OUT, "librpkt_gen.so")
# the engine: one translation unit per kernel family, shared device code in rpkt_common.h
GPU_SRC = [os.path.join(HERE, "csrc", f) for f in
           ("rpkt_parse.hip", "rpkt_tx.hip", "rpkt_walks.hip", "rpkt_fields.hip", "rpkt_tunnel.hip",
            "rpkt_abi.hip", "rpkt_coll.hip")]
GPU_DEPS = [os.path.join(HERE, "csrc", "rpkt_common.h"), os.path.join(HERE, "csrc", "rpkt_opts.h"),
            os.path.join(HERE, "csrc", "rpkt_proto_table.h")]        # included; the table is generated
# units compiled a second time with other defines (same source: same unit hash)
SECOND_COMPILES = [("rpkt_tx.hip", "rpkt_tx_w64.o", ["-DRPKT_WIN=64", "-DRPKT_TX_W64"]),
                   # only the compact parse of short strided frames: the unit's other
                   # kernels are not used by this compile
                   ("rpkt_parse.hip", "rpkt_parse_w64.o", ["-DRPKT_WIN=64", "-DRPKT_PARSE_W64",
                                                           "-Wno-unused-function",
                                                           "-Wno-unused-const-variable",
                                                           "-Wno-unneeded-internal-declaration"])]
# the csrc headers each unit includes (directly or through another header): a unit's
# hash covers these, so a change to the option walks' header leaves tx / fields profiles valid
UNIT_HEADERS = {"rpkt_parse.hip": ("rpkt_common.h", "rpkt_opts.h"),
                "rpkt_tx.hip": ("rpkt_common.h",),
                "rpkt_walks.hip": ("rpkt_common.h", "rpkt_opts.h", "rpkt_proto_table.h"),
                "rpkt_fields.hip": ("rpkt_common.h",),
                "rpkt_tunnel.hip": ("rpkt_common.h",),
                "rpkt_abi.hip": ("rpkt_common.h",),
                "rpkt_coll.hip": ("rpkt_common.h",)}
# every unit has its header list (a unit added to GPU_SRC without one would make
# source_hash raise at the first build: fail here, at import, instead)
assert set(UNIT_HEADERS) == {os.path.basename(f) for f in GPU_SRC}, "UNIT_HEADERS vs GPU_SRC"
GEN_SRC = [os.path.join(HERE, "csrc", "rpkt_gen.cpp")]
HDR = [os.path.join(ROOT, "include", "rpkt_gpu.h"), os.path.join(ROOT, "include", "rpkt_protocols.h")]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def source_hash(units=None, defines=()):
    """Short hash of the engine sources (or of some units plus the shared headers) and of
    the compile-time switches they are built with (`defines`, e.g. an ablation build's
    -DRPKT_IP6_DIST=0): ties profiles/ numbers to a kernel build."""
    import hashlib
    h = hashlib.sha1()
    if defines:
        h.update(("\0".join(defines) + "\0").encode())
    srcs = GPU_SRC if units is None else [f for f in GPU_SRC if os.path.basename(f) in units]
    deps = GPU_DEPS
    if units is not None:                  # the headers those units include
        deps = [d for d in GPU_DEPS if any(os.path.basename(d) in UNIT_HEADERS[u] for u in units)]
    for f in srcs + deps + HDR:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:12]


def unit_hashes(defines=()):
    """Per-unit hashes (unit file + shared headers + compile switches), so a profile of one
    kernel family stays valid while another unit changes: "parse=... tx=... walks=..."."""
    return " ".join("%s=%s" % (u, source_hash(["rpkt_%s.hip" % u], defines))
                    for u in ("parse", "tx", "walks", "fields", "tunnel"))


def build_gpu(force=False, extra=()):
    """Compile the units in parallel (hipcc -c, gfx950), then link the product library and
    the development library (-DRPKT_ABLATE)."""
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(OUT, exist_ok=True)
    deps = GPU_SRC + GPU_DEPS + HDR + [os.path.abspath(__file__)]   # the flags and hashes too
    if not (force or _stale(GPU_LIB, deps) or _stale(ABLATE_LIB, deps)):
        return GPU_LIB
    defines = tuple(x for x in extra if x.startswith("-D"))
    flags = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wall",
             '-DRPKT_SRC_HASH="%s"' % source_hash(None, defines),
             '-DRPKT_UNIT_HASHES="%s"' % unit_hashes(defines)] + list(extra)
    units = [(f, os.path.basename(f)[:-4], []) for f in GPU_SRC]
    units += [(os.path.join(HERE, "csrc", src), obj[:-2], d) for src, obj, d in SECOND_COMPILES]
    libs = {GPU_LIB: [], ABLATE_LIB: []}
    jobs = []
    for src, stem, d in units:
        for lib, sfx, dd in ((GPU_LIB, "", []), (ABLATE_LIB, "_ablate", ["-DRPKT_ABLATE"])):
            obj = os.path.join(OUT, stem + sfx + ".o")
            jobs.append((src, obj, d + dd))
            libs[lib].append(obj)
    with ThreadPoolExecutor(max_workers=min(len(jobs), 8)) as ex:
        list(ex.map(lambda j: subprocess.check_call(flags + j[2] + ["-c", "-o", j[1], j[0]]), jobs))
    # RCCL is not linked: rpkt_coll.hip resolves it on first use (the copy already in the
    # process first, so under torch the communicator and the library match)
    for lib, objs in libs.items():
        subprocess.check_call([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] +
                              objs + ["-ldl"])
    return GPU_LIB


def build_gen(force=False):
    os.makedirs(OUT, exist_ok=True)
    if force or _stale(GEN_LIB, GEN_SRC):
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-o", GEN_LIB] + \
            GEN_SRC + ["-lpthread"]
        subprocess.check_call(cmd)
    return GEN_LIB


EXAMPLES = ("parse_batch", "flow_reduce", "rx_graph", "vtep_rx")
EXAMPLE_BIN = os.path.join(ROOT, "examples", "parse_batch")
FLOW_REDUCE_BIN = os.path.join(ROOT, "examples", "flow_reduce")
VTEP_RX_BIN = os.path.join(ROOT, "examples", "vtep_rx")


def build_example(force=False):
    """The C++ host examples: link librpkt_gpu.so through the C ABI only (and RCCL for
    the communicator flow_reduce makes)."""
    out = []
    for name in EXAMPLES:
        src = os.path.join(ROOT, "examples", name + ".cpp")
        binp = os.path.join(ROOT, "examples", name)
        if force or _stale(binp, [src, GPU_LIB] + HDR):
            cmd = [HIPCC, "-O2", "-I" + os.path.join(ROOT, "include"), src, "-L" + OUT,
                   "-lrpkt_gpu", "-L" + ROCM_LIB, "-lrccl",
                   "-Wl,-rpath,$ORIGIN/../rpkt_amd/_build", "-o", binp]
            subprocess.check_call(cmd)
        out.append(binp)
    return out


def build_all(force=False):
    return build_gpu(force), build_gen(force), build_example(force)


if __name__ == "__main__":
    import sys
    print(build_all(force="--force" in sys.argv))
