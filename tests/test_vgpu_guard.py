"""The container-side tier of a time-sliced share (Gaia two-tier vGPU, paper p.3 §III.A):
``libgtk_vgpu.so`` preloaded into a pod caps every HIP allocation at the share's HBM and forces the
share's HSA_CU_MASK whatever the container's environment says.  CPU tests run it against a stand-in
HIP runtime named ``libamdhip64.so`` (csrc/vgpu/fake_hip.cpp), loaded both ways a real process loads
HIP: RTLD_LOCAL (the PyTorch wheel's bundled runtime, found by the guard's fallback lookup) and
RTLD_GLOBAL (found by RTLD_NEXT)."""
import json
import os
import subprocess
import sys

import pytest

from gpu_topology_on_k8s_amd._native import binary

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GiB = 1 << 30

CHILD = r"""
import ctypes, json, os, sys
mode = ctypes.RTLD_GLOBAL if sys.argv[2] == "global" else ctypes.RTLD_LOCAL
rt = ctypes.CDLL(sys.argv[1], mode=mode)       # the 'HIP runtime' the application links
glob = ctypes.CDLL(None)
def sym(name):                                 # as the application resolves a symbol: global scope first
    try:
        return getattr(glob, name)
    except AttributeError:
        return getattr(rt, name)
vp = ctypes.c_void_p
class Extent(ctypes.Structure):
    _fields_ = [("width", ctypes.c_size_t), ("height", ctypes.c_size_t), ("depth", ctypes.c_size_t)]
class Pitched(ctypes.Structure):
    _fields_ = [("ptr", vp), ("pitch", ctypes.c_size_t), ("xsize", ctypes.c_size_t), ("ysize", ctypes.c_size_t)]
def malloc(n, fn="hipMalloc"):
    p = vp()
    if fn == "hipMallocPitch":
        pitch = ctypes.c_size_t()
        return sym(fn)(ctypes.byref(p), ctypes.byref(pitch), ctypes.c_size_t(n), ctypes.c_size_t(1)), p
    if fn == "hipMalloc3D":
        pp = Pitched()
        e = sym(fn)(ctypes.byref(pp), Extent(1 << 20, n >> 20, 1))  # n bytes as 1 MiB rows (pitch = width)
        return e, vp(pp.ptr)
    args = {"hipMalloc": (), "hipExtMallocWithFlags": (ctypes.c_uint(0),), "hipMallocManaged": (ctypes.c_uint(1),),
            "hipMallocAsync": (vp(),), "hipHostMalloc": (ctypes.c_uint(0),)}[fn]
    return sym(fn)(ctypes.byref(p), ctypes.c_size_t(n), *args), p
GiB = 1 << 30
out = {"env_mask": os.environ.get("HSA_CU_MASK"), "active": os.environ.get("GTK_VGPU_ACTIVE")}
e1, p1 = malloc(6 * GiB)
e2, p2 = malloc(3 * GiB, "hipExtMallocWithFlags")    # 6 + 3 > 8: refused
e3, p3 = malloc(2 * GiB, "hipMallocManaged")
glob.gtk_vgpu_used.restype = ctypes.c_longlong
used_after = glob.gtk_vgpu_used(0)
free_, total = ctypes.c_size_t(), ctypes.c_size_t()
sym("hipMemGetInfo")(ctypes.byref(free_), ctypes.byref(total))
e7, p7 = malloc(1 * GiB, "hipMalloc3D")              # the share is full: 3D arrays are refused too
e8, p8 = malloc(40 * GiB, "hipHostMalloc")           # host memory is not the share's
h = vp()
e9 = sym("hipMemCreate")(ctypes.byref(h), ctypes.c_size_t(1 << 20), None, ctypes.c_ulonglong(0))  # VMM: counted
sym("hipFree")(p1)
sym("hipMemRelease")(h)
e4, p4 = malloc(5 * GiB, "hipMallocAsync")          # fits again once 6 GiB came back
e5, p5 = malloc(1 << 20, "hipMallocPitch")
e10, p10 = malloc(1 * GiB - (1 << 20), "hipMalloc3D")  # and a 3D array up to the share
os.environ["FAKE_HIP_DEVICE"] = "1"                 # no limit configured on ordinal 1
e6, p6 = malloc(40 * GiB)
out.update(e=[e1, e2, e3, e4, e5, e6], e3d=[e7, e10], host=e8, vmm=e9, p2_null=not p2.value, used_after=used_after,
           free=free_.value, total=total.value, used_end=glob.gtk_vgpu_used(0))
print(json.dumps(out))
"""


def _fake():
    return os.path.join(os.path.dirname(str(binary("libgtk_vgpu.so"))), "fake_hip", "libamdhip64.so")


def _run(tmp_path, mode, config=True, env_mask="0:0-255"):
    fake = _fake()
    conf = tmp_path / "gtk-vgpu.conf"
    if config:
        conf.write_text(f"# written by the device plugin at Allocate\nhbm_limit 0 {8 * GiB}\ncu_mask 0:64-127\n")
    env = dict(os.environ, GTK_VGPU_CONFIG=str(conf), HSA_CU_MASK=env_mask, FAKE_HIP_DEVICE="0")
    guard = str(binary("libgtk_vgpu.so"))
    env["LD_PRELOAD"] = (env["LD_PRELOAD"] + ":" if env.get("LD_PRELOAD") else "") + guard  # keep what is preloaded already
    p = subprocess.run([sys.executable, "-c", CHILD, fake, mode], capture_output=True, text=True, timeout=60, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("mode", ["local", "global"])
def test_guard_caps_hbm_and_forces_the_cu_mask(tmp_path, mode):
    """Accounting at ROCr's pool allocator: every HIP allocation path (hipMalloc, ...WithFlags,
    Managed, Async, Pitch, 3D, hipMemCreate) is charged once, host memory is not, and a refusal
    surfaces as HIP's hipErrorOutOfMemory."""
    out = _run(tmp_path, mode)
    assert out["active"] == "1" and out["env_mask"] == "0:64-127"  # the container's own value is overridden
    e1, e2, e3, e4, e5, e6 = out["e"]
    assert e1 == 0 and e2 == 2 and out["p2_null"]  # hipErrorOutOfMemory past the share
    assert e3 == 0 and out["used_after"] == 8 * GiB  # exactly at the share is fine
    assert out["total"] == 8 * GiB and out["free"] == 0  # hipMemGetInfo reports the share
    assert out["e3d"] == [2, 0]  # hipMalloc3D past the share is refused; within it, granted
    assert out["host"] == 0 and out["vmm"] == 2  # host pools are not counted; a full share refuses VMM too
    assert e4 == 0 and e5 == 0 and e6 == 0  # freed memory returns; other ordinals are not limited
    # 2 (managed) + 5 (async) GiB + one pitched 1 MiB row + a 1 GiB - 1 MiB 3D array
    assert out["used_end"] == 8 * GiB


REWRITE_CHILD = r"""
import ctypes, json, os, sys
os.environ["HSA_CU_MASK"] = "0:0-255"          # the program rewrites the mask before any HIP call
rt = ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_GLOBAL if sys.argv[2] == "global" else ctypes.RTLD_LOCAL)
n = ctypes.c_int()
first = sys.argv[3]
if first == "hipDeviceGetAttribute":
    rt.hipDeviceGetAttribute(ctypes.byref(n), ctypes.c_int(0), ctypes.c_int(0))
else:
    getattr(rt, first)(*([ctypes.byref(n)] if first in ("hipGetDeviceCount", "hipGetDevice", "hipRuntimeGetVersion")
                         else [ctypes.c_int(0)]))
rt.fake_hip_init_mask.restype = ctypes.c_char_p
rt.fake_hip_stream_mask.restype = ctypes.c_char_p
s1, s2, s3 = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
rt.hipStreamCreate(ctypes.byref(s1))
every = (ctypes.c_uint32 * 8)(*([0xFFFFFFFF] * 8))                 # a stream asking for all 256 CUs
rt.hipExtStreamCreateWithCUMask(ctypes.byref(s2), ctypes.c_uint32(8), every)
part = (ctypes.c_uint32 * 8)(*([0xFFFFFFFF] * 3 + [0] * 5))        # ... for CUs 0-95
rt.hipExtStreamCreateWithCUMask(ctypes.byref(s3), ctypes.c_uint32(8), part)
s4 = ctypes.c_void_p()
low = (ctypes.c_uint32 * 8)(*([0xFFFFFFFF] + [0] * 7))             # ... for CUs 0-31, none of them the share's
rt.hipExtStreamCreateWithCUMask(ctypes.byref(s4), ctypes.c_uint32(8), low)
print(json.dumps({"init_mask": rt.fake_hip_init_mask().decode(),
                  "queues": [rt.fake_hip_stream_mask(s).decode() for s in (s1, s2, s3, s4)]}))
"""


@pytest.mark.parametrize("mode,first", [("local", "hipGetDeviceCount"), ("global", "hipSetDevice"), ("local", "hipGetDevice"),
                                        ("local", "hipRuntimeGetVersion"), ("global", "hipDeviceGetAttribute")])
def test_guard_enforces_the_mask_at_rocr_whatever_the_first_call(tmp_path, mode, first):
    """A program that rewrites HSA_CU_MASK in its own environment after the guard's constructor ran,
    whatever its first HIP call: ROCr initialises with the share's mask (set back in hsa_init), every
    queue runs on the share's CUs, and a stream's own CU mask is narrowed to the share (VERDICT r3
    next #5).  Without the guard the runtime reads the program's value and queues get every CU."""
    fake = _fake()
    conf = tmp_path / "gtk-vgpu.conf"
    conf.write_text(f"hbm_limit 0 {8 * GiB}\ncu_mask 0:64-127\n")
    env = dict(os.environ, GTK_VGPU_CONFIG=str(conf), FAKE_HIP_DEVICE="0")
    guard = str(binary("libgtk_vgpu.so"))
    env["LD_PRELOAD"] = (env["LD_PRELOAD"] + ":" if env.get("LD_PRELOAD") else "") + guard
    p = subprocess.run([sys.executable, "-c", REWRITE_CHILD, fake, mode, first], capture_output=True, text=True, timeout=60,
                       env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["init_mask"] == "0:64-127"
    # a stream mask with no CU of the share would stop its queue: the share's own mask applies instead
    assert out["queues"] == ["64-127", "64-127", "64-95", "64-127"]
    env.pop("LD_PRELOAD")
    q = subprocess.run([sys.executable, "-c", REWRITE_CHILD, fake, mode, first], capture_output=True, text=True, timeout=60,
                       env=env)
    assert q.returncode == 0, q.stderr[-2000:]
    out = json.loads(q.stdout.strip().splitlines()[-1])
    assert out["init_mask"] == "0:0-255" and out["queues"] == ["0-255", "0-255", "0-95", "0-31"]


RENUMBER_CHILD = r"""
import ctypes, json, os, sys
rt = ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_LOCAL)
g = ctypes.CDLL(None)
GiB = 1 << 30
def alloc(n, fn="hipMalloc"):
    p = ctypes.c_void_p()
    args = (ctypes.c_uint(1),) if fn == "hipMallocManaged" else ()
    f = getattr(g, fn) if hasattr(g, fn) else getattr(rt, fn)  # global scope first, as the application links
    return f(ctypes.byref(p), ctypes.c_size_t(n), *args), p
n = ctypes.c_int()
rt.hipGetDeviceCount(ctypes.byref(n))
bus = ctypes.create_string_buffer(64)
rt.hipDeviceGetPCIBusId(bus, 64, 0)
e1, p1 = alloc(6 * GiB)
e2, p2 = alloc(3 * GiB, "hipMallocManaged")   # managed memory (system pages here, as with HMM) is charged too
e3, p3 = alloc(2 * GiB, "hipMallocManaged")
g.gtk_vgpu_used.restype = ctypes.c_longlong
used_full = g.gtk_vgpu_used(g.gtk_vgpu_hip_ordinal(0))
free_, total = ctypes.c_size_t(), ctypes.c_size_t()
g.hipMemGetInfo(ctypes.byref(free_), ctypes.byref(total))
g.hipFree(p3)                                   # ... and given back by hipFree
used_freed = g.gtk_vgpu_used(g.gtk_vgpu_hip_ordinal(0))
s = ctypes.c_void_p()
rt.hipStreamCreate(ctypes.byref(s))
rt.fake_hip_init_mask.restype = ctypes.c_char_p
rt.fake_hip_stream_mask.restype = ctypes.c_char_p
out = {"count": n.value, "bus0": bus.value.decode(), "e": [e1, e2, e3], "used_full": used_full, "used_freed": used_freed,
       "total": total.value, "free": free_.value, "queue": rt.fake_hip_stream_mask(s).decode(),
       "init_mask": rt.fake_hip_init_mask().decode(), "rocr_ordinal": g.gtk_vgpu_hip_ordinal(0)}
if n.value > 1:                                 # the other GPU is not the share's
    os.environ["FAKE_HIP_DEVICE"] = "1"
    out["other"] = alloc(40 * GiB)[0]
print(json.dumps(out))
"""


@pytest.mark.parametrize("visible,rocr_ordinal", [({}, 1), ({"ROCR_VISIBLE_DEVICES": "1,0"}, 0),
                                                  ({"HIP_VISIBLE_DEVICES": "1"}, 1), ({"ROCR_VISIBLE_DEVICES": "1"}, 0)])
def test_address_keyed_share_holds_under_renumbering(tmp_path, visible, rocr_ordinal):
    """ADVICE r4 (vgpu_guard.cpp ordinal keying): the plugin names the share's GPU by PCI address, so
    a pod that reorders or hides devices with $ROCR_VISIBLE_DEVICES / $HIP_VISIBLE_DEVICES cannot move
    its limit or mask onto another GPU.  The share is physical GPU 1 (0000:15:00.0); whichever HIP
    number it ends up with, its allocations are capped, hipMemGetInfo reports the share, its queues
    run on the share's CUs (an ordinal-keyed HSA_CU_MASK in the pod's environment is cleared), and the
    other GPU, when visible, is not limited.  Managed allocations, which do not reach a device pool
    here (system memory, as with HMM), are charged at the HIP level and released by hipFree."""
    conf = tmp_path / "gtk-vgpu.conf"
    conf.write_text(f"hbm_limit_bdf 0000:15:00.0 {8 * GiB}\ncu_mask_bdf 0000:15:00.0 64-127\n")
    hip0_is_share = visible != {}
    env = {k: v for k, v in os.environ.items() if k not in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES")}
    env.update(GTK_VGPU_CONFIG=str(conf), HSA_CU_MASK="0:0-255", FAKE_HIP_DEVICE="0" if hip0_is_share else "1", **visible)
    env["LD_PRELOAD"] = (env["LD_PRELOAD"] + ":" if env.get("LD_PRELOAD") else "") + str(binary("libgtk_vgpu.so"))
    child = RENUMBER_CHILD if hip0_is_share else RENUMBER_CHILD.replace("(bus, 64, 0)", "(bus, 64, 1)").replace(
        "hip_ordinal(0)", "hip_ordinal(1)").replace('os.environ["FAKE_HIP_DEVICE"] = "1"', 'os.environ["FAKE_HIP_DEVICE"] = "0"')
    p = subprocess.run([sys.executable, "-c", child, _fake()], capture_output=True, text=True, timeout=60, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["bus0"] == "0000:15:00.0", out
    assert out["e"] == [0, 2, 0] and out["used_full"] == 8 * GiB and out["used_freed"] == 6 * GiB, out
    assert out["total"] == 8 * GiB and out["free"] == 0, out
    assert out["queue"] == "64-127" and out["init_mask"] == "", out
    assert out["rocr_ordinal"] == rocr_ordinal, out
    if out["count"] > 1:
        assert out["other"] == 0, out


def test_pool_backed_managed_memory_is_charged_once(tmp_path):
    """A runtime without HMM backs hipMallocManaged with a device pool: the pool hook charges the block,
    and the HIP-level managed hook sees that and does not charge it a second time (which would refuse
    a block that fits: 6 GiB + 2 GiB managed in an 8 GiB share)."""
    conf = tmp_path / "gtk-vgpu.conf"
    conf.write_text(f"hbm_limit_bdf 0000:15:00.0 {8 * GiB}\ncu_mask_bdf 0000:15:00.0 64-127\n")
    env = {k: v for k, v in os.environ.items() if k not in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES")}
    env.update(GTK_VGPU_CONFIG=str(conf), FAKE_HIP_DEVICE="1", FAKE_HIP_MANAGED_IN_POOL="1")
    env["LD_PRELOAD"] = (env["LD_PRELOAD"] + ":" if env.get("LD_PRELOAD") else "") + str(binary("libgtk_vgpu.so"))
    child = RENUMBER_CHILD.replace("(bus, 64, 0)", "(bus, 64, 1)").replace("hip_ordinal(0)", "hip_ordinal(1)").replace(
        'os.environ["FAKE_HIP_DEVICE"] = "1"', 'os.environ["FAKE_HIP_DEVICE"] = "0"')
    p = subprocess.run([sys.executable, "-c", child, _fake()], capture_output=True, text=True, timeout=60, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["e"] == [0, 2, 0] and out["used_full"] == 8 * GiB and out["used_freed"] == 6 * GiB, out


def test_introspection_before_the_runtime_starts_does_not_disable_the_share(tmp_path):
    """The guard's address-keyed config is resolved once ROCr can enumerate its agents.  A call into
    the guard before the runtime is initialised (here its exported introspection entry point, first
    thing in the process) must not freeze an empty enumeration: the share still holds afterwards."""
    conf = tmp_path / "gtk-vgpu.conf"
    conf.write_text(f"hbm_limit_bdf 0000:15:00.0 {8 * GiB}\ncu_mask_bdf 0000:15:00.0 64-127\n")
    env = {k: v for k, v in os.environ.items() if k not in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES")}
    env.update(GTK_VGPU_CONFIG=str(conf), FAKE_HIP_DEVICE="0", ROCR_VISIBLE_DEVICES="1,0")
    env["LD_PRELOAD"] = (env["LD_PRELOAD"] + ":" if env.get("LD_PRELOAD") else "") + str(binary("libgtk_vgpu.so"))
    early = ("import ctypes\ng0 = ctypes.CDLL(None)\ng0.gtk_vgpu_limit.restype = ctypes.c_longlong\n"
             "early = (g0.gtk_vgpu_hip_ordinal(0), g0.gtk_vgpu_limit(0))\n")
    child = early + RENUMBER_CHILD.replace('"rocr_ordinal": g.gtk_vgpu_hip_ordinal(0)}', '"rocr_ordinal": g.gtk_vgpu_hip_ordinal(0), "early": early}')
    p = subprocess.run([sys.executable, "-c", child, _fake()], capture_output=True, text=True, timeout=60, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["early"] == [0, -1], out  # before the runtime: unresolved (HIP number, no limit yet)
    assert out["e"] == [0, 2, 0] and out["total"] == 8 * GiB and out["queue"] == "64-127", out


def test_ordinal_keyed_share_moves_with_renumbering(tmp_path):
    """Why the plugin writes addresses: the same share keyed by ordinal 0 lands on whichever GPU the
    pod's own ROCR_VISIBLE_DEVICES puts first -- here the other one, and the share's GPU is uncapped."""
    conf = tmp_path / "gtk-vgpu.conf"
    conf.write_text(f"hbm_limit 0 {8 * GiB}\n")
    env = {k: v for k, v in os.environ.items() if k not in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES")}
    env.update(GTK_VGPU_CONFIG=str(conf), FAKE_HIP_DEVICE="1", ROCR_VISIBLE_DEVICES="1,0")
    env["LD_PRELOAD"] = (env["LD_PRELOAD"] + ":" if env.get("LD_PRELOAD") else "") + str(binary("libgtk_vgpu.so"))
    child = RENUMBER_CHILD.replace("(bus, 64, 0)", "(bus, 64, 1)")
    p = subprocess.run([sys.executable, "-c", child, _fake()], capture_output=True, text=True, timeout=60, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["bus0"] == "0000:05:00.0" and out["e"] == [0, 0, 0], out  # physical GPU 0, the plugin's "ordinal 0": uncapped


def test_mounted_config_wins_over_the_pods_environment(tmp_path):
    """ADVICE r3 (vgpu_guard.cpp:322): a pod spec that points GTK_VGPU_CONFIG elsewhere does not make
    the guard inert when the plugin's config is mounted: the fixed mount path is read first.  (The
    mount path is a compile-time constant; this builds the guard with it pointed into tmp_path.)"""
    fixed = tmp_path / "fixed.conf"
    fixed.write_text(f"hbm_limit 0 {8 * GiB}\ncu_mask 0:64-127\n")
    lib = tmp_path / "libgtk_vgpu_fixed.so"
    src = os.path.join(REPO, "csrc", "vgpu", "vgpu_guard.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-shared", "-fPIC", "-fvisibility=hidden", "-I/opt/rocm/include",
                    f'-DGTK_VGPU_FIXED_CONF="{fixed}"', src, "-o", str(lib), "-ldl", "-pthread"], check=True, timeout=120)
    env = dict(os.environ, GTK_VGPU_CONFIG="/nonexistent", HSA_CU_MASK="0:0-255", FAKE_HIP_DEVICE="0")
    env["LD_PRELOAD"] = (env["LD_PRELOAD"] + ":" if env.get("LD_PRELOAD") else "") + str(lib)
    p = subprocess.run([sys.executable, "-c", CHILD, _fake(), "local"], capture_output=True, text=True, timeout=60, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["active"] == "1" and out["env_mask"] == "0:64-127" and out["e"][1] == 2


def test_guard_without_config_is_a_pass_through(tmp_path):
    out = _run(tmp_path, "local", config=False)
    assert out["active"] is None and out["env_mask"] == "0:0-255"
    assert out["e"] == [0, 0, 0, 0, 0, 0] and out["e3d"] == [0, 0] and out["vmm"] == 0 and out["total"] == 64 * GiB


def test_allocate_mounts_the_guard_for_a_partial_gpu_only():
    """Through the cluster: a 0.5-GPU pod on a 4-slice node gets the guard library and its config
    mounted read-only and preloaded; the config caps ordinal 0 at its two slices' HBM and carries the
    same CU mask as the env; a pod holding whole GPUs' worth of slices gets no guard."""
    from gpu_topology_on_k8s_amd.k8s import Contract
    from gpu_topology_on_k8s_amd.sim import SimCluster
    from gpu_topology_on_k8s_amd.topology import fixtures as fx
    from gpu_topology_on_k8s_amd.topology.shares import time_slice

    C = Contract()
    v = time_slice(fx.f7_mi355x(n=2), 4)
    with SimCluster({"s": v}) as c:
        c.submit("half", 2, slices=True, annotations={C.fraction_key: "0.5"})
        r = c.schedule_pending()[0]
        assert r.node == "s", r
        resp = c.nodes["s"].kubelet.responses["default/half"].container_responses[0]
        envs = dict(resp.envs)
        mounts = {m.container_path: (m.host_path, m.read_only) for m in resp.mounts}
        assert envs["LD_PRELOAD"] == "/usr/local/lib/gtk-vgpu/libgtk_vgpu.so" and envs["GTK_VGPU_CONFIG"] == "/etc/gtk-vgpu.conf"
        lib, ro = mounts["/usr/local/lib/gtk-vgpu/libgtk_vgpu.so"]
        assert ro and os.path.getsize(lib) == os.path.getsize(str(binary("libgtk_vgpu.so")))
        conf, ro = mounts["/etc/gtk-vgpu.conf"]
        text = open(conf).read()
        # keyed by PCI address, the CUs the same as the env's mask for that GPU
        bdf = envs["GTK_GPU_BDFS"].split(",")[0]
        assert ro and f"hbm_limit_bdf {bdf} {2 * (288_000_000_000 // 4)}" in text, text
        ordinal, cus = envs["HSA_CU_MASK"].split(":")
        assert ordinal == "0" and f"cu_mask_bdf {bdf} {cus}" in text and "hbm_limit 0" not in text, text
        acct, ro = mounts["/var/run/gtk-vgpu.acct"]  # the pod's shared budget, writable by any container user
        assert not ro and "acct /var/run/gtk-vgpu.acct" in text and os.stat(acct).st_mode & 0o666 == 0o666
        c.submit("whole", 4, slices=True)  # a whole GPU's worth of slices: no share to guard
        r = c.schedule_pending()[0]
        resp = c.nodes["s"].kubelet.responses["default/whole"].container_responses[0]
        assert r.node == "s" and not resp.mounts and "LD_PRELOAD" not in dict(resp.envs)
        assert "gtk_plugin_guarded_containers_total 1.0" in c.nodes["s"].plugin.metrics.exposition().decode()


def test_plugin_config_caps_the_share_whatever_the_pod_renumbers(tmp_path):
    """The plugin's own config for half of physical GPU 1 (slices 4, 5), read by the guard in a process
    whose ROCR_VISIBLE_DEVICES puts that GPU first: the share's GPU is capped and masked; without an
    address (discovery found none) the config falls back to ordinals."""
    import dataclasses

    from gpu_topology_on_k8s_amd.deviceplugin import DevicePluginServer, PluginConfig
    from gpu_topology_on_k8s_amd.topology import fixtures as fx
    from gpu_topology_on_k8s_amd.topology.shares import time_slice

    v = time_slice(fx.f7_mi355x(n=2), 4)
    plug = DevicePluginServer(v, PluginConfig(device_specs="stub", dev_root=str(tmp_path), share_guard="env",
                                              guard_dir=str(tmp_path / "g")))
    from gpu_topology_on_k8s_amd.topology.shares import cu_mask_env

    text = plug.guard_config([4, 5], cu_mask_env(v, [4, 5]), acct=False)
    assert "hbm_limit_bdf 0000:15:00.0 " in text and "cu_mask_bdf 0000:15:00.0 0-127" in text, text
    conf = tmp_path / "gtk-vgpu.conf"
    conf.write_text(text.replace(f" {2 * (288_000_000_000 // 4)}", f" {8 * GiB}"))
    env = {k: val for k, val in os.environ.items() if k not in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES")}
    env.update(GTK_VGPU_CONFIG=str(conf), HSA_CU_MASK="0:0-255", FAKE_HIP_DEVICE="0", ROCR_VISIBLE_DEVICES="1,0")
    env["LD_PRELOAD"] = (env["LD_PRELOAD"] + ":" if env.get("LD_PRELOAD") else "") + str(binary("libgtk_vgpu.so"))
    p = subprocess.run([sys.executable, "-c", RENUMBER_CHILD, _fake()], capture_output=True, text=True, timeout=60, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["e"] == [0, 2, 0] and out["total"] == 8 * GiB and out["queue"] == "0-127" and out["other"] == 0, out
    bare = dataclasses.replace(v, gpus=[dataclasses.replace(g, bdf="") for g in v.gpus])
    plug2 = DevicePluginServer(bare, PluginConfig(device_specs="stub", dev_root=str(tmp_path), share_guard="env",
                                                  guard_dir=str(tmp_path / "g2")))
    text = plug2.guard_config([4, 5], cu_mask_env(bare, [4, 5]), acct=False)
    assert "hbm_limit 0 " in text and "cu_mask 0:0-127" in text and "_bdf" not in text, text


def test_preload_mode_mounts_ld_so_preload(tmp_path):
    from gpu_topology_on_k8s_amd.deviceplugin import DevicePluginServer, PluginConfig
    from gpu_topology_on_k8s_amd.topology import fixtures as fx
    from gpu_topology_on_k8s_amd.topology.shares import time_slice

    v = time_slice(fx.f7_mi355x(n=2), 4)
    plug = DevicePluginServer(v, PluginConfig(device_specs="stub", dev_root=str(tmp_path), share_guard="preload",
                                              guard_dir=str(tmp_path / "g")))
    assert plug.install_guard()
    r = plug._container_response([0], {})
    mounts = {m.container_path: m.host_path for m in r.mounts}
    assert open(mounts["/etc/ld.so.preload"]).read().strip() == "/usr/local/lib/gtk-vgpu/libgtk_vgpu.so"
    assert dict(r.envs)["LD_PRELOAD"] == "/usr/local/lib/gtk-vgpu/libgtk_vgpu.so"
    whole = DevicePluginServer(fx.f7_mi355x(n=2), PluginConfig(share_guard="env", guard_dir=str(tmp_path / "w")))
    assert whole.install_guard() is False  # whole-GPU nodes: nothing to guard


HOLDER = r"""
import ctypes, sys
rt = ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_LOCAL)
p = ctypes.c_void_p()
print(rt.hipMalloc(ctypes.byref(p), ctypes.c_size_t(6 << 30)), flush=True)
sys.stdin.readline()          # hold the 6 GiB until told to go; exit WITHOUT freeing (a crash)
"""

PROBE = r"""
import ctypes, json, sys
rt = ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_LOCAL)
g = ctypes.CDLL(None)
g.gtk_vgpu_pod_used.restype = ctypes.c_longlong
res = []
for n in [int(x) for x in sys.argv[2].split(",")]:
    p = ctypes.c_void_p()
    res.append(rt.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n << 30)))
free_, total = ctypes.c_size_t(), ctypes.c_size_t()
g.hipMemGetInfo(ctypes.byref(free_), ctypes.byref(total))
print(json.dumps({"e": res, "pod_used": g.gtk_vgpu_pod_used(0), "free": free_.value}))
"""


def test_pod_wide_budget_across_processes_and_crash_release(tmp_path):
    """With an ``acct`` file every process of the pod draws from one budget; a process that dies
    holding memory gives it back (its slot lock dies with it)."""
    fake = os.path.join(os.path.dirname(str(binary("libgtk_vgpu.so"))), "fake_hip", "libamdhip64.so")
    conf = tmp_path / "gtk-vgpu.conf"
    conf.write_text(f"hbm_limit 0 {8 * GiB}\nacct {tmp_path / 'pod.acct'}\n")
    env = dict(os.environ, GTK_VGPU_CONFIG=str(conf), FAKE_HIP_DEVICE="0")
    env["LD_PRELOAD"] = (env["LD_PRELOAD"] + ":" if env.get("LD_PRELOAD") else "") + str(binary("libgtk_vgpu.so"))
    holder = subprocess.Popen([sys.executable, "-c", HOLDER, fake], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env)
    try:
        assert holder.stdout.readline().strip() == "0"  # 6 of 8 GiB taken by another process of the pod
        p = subprocess.run([sys.executable, "-c", PROBE, fake, "3,2"], capture_output=True, text=True, timeout=60, env=env)
        assert p.returncode == 0, p.stderr
        out = json.loads(p.stdout.strip().splitlines()[-1])
        assert out["e"] == [2, 0] and out["pod_used"] == 8 * GiB and out["free"] == 0
    finally:
        holder.stdin.write("go\n")
        holder.stdin.flush()
        holder.wait(timeout=30)
    p = subprocess.run([sys.executable, "-c", PROBE, fake, "5"], capture_output=True, text=True, timeout=60, env=env)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["e"] == [0] and out["pod_used"] == 5 * GiB  # the dead processes' bytes are gone


@pytest.mark.parametrize("sanitizer", ["tsan", "asan"])
@pytest.mark.parametrize("pod_wide,keyed", [(False, "ordinal"), (True, "ordinal"), (False, "bdf"), (True, "bdf")])
def test_guard_under_sanitizers(tmp_path, sanitizer, pod_wide, keyed):
    """SURVEY.md §5.2 for the guard: 16 threads allocating and freeing against one budget (and, pod-wide,
    a forked child drawing from the parent's budget) under ThreadSanitizer and ASan/UBSan — no race, no
    memory error, never past the limit, every byte returned; pool and managed allocations mixed, the
    device named by ordinal or by PCI address (resolved concurrently with the first allocations).  (TSan found two races in the first
    version: a lazily resolved entry point, and an address reused between the runtime's free and the
    guard forgetting it.)"""
    exe = str(binary(f"vgpu_selftest_{sanitizer}"))
    conf = tmp_path / "c.conf"
    limit = f"hbm_limit 0 {8 * GiB}" if keyed == "ordinal" else f"hbm_limit_bdf 0000:05:00.0 {8 * GiB}"
    conf.write_text(limit + "\n" + (f"acct {tmp_path / 'pod.acct'}\n" if pod_wide else ""))
    env = dict(os.environ, GTK_VGPU_CONFIG=str(conf))
    if pod_wide:
        env["SELFTEST_ACCT"] = "1"
    p = subprocess.run([exe, "16", "1500"], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, (p.stdout[-1000:], p.stderr[-4000:])
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["ok"] > 0 and out["oom"] > 0


def test_training_entry_does_not_cap_twice_under_the_guard(monkeypatch):
    """torch's memory fraction is taken of hipMemGetInfo's total, which the guard already reports as
    the share: with the guard in force the cooperative cap must not be applied on top of it."""
    import torch

    from gpu_topology_on_k8s_amd.models import train as tr

    calls = []
    monkeypatch.setattr(torch.cuda, "set_per_process_memory_fraction", lambda f, d: calls.append((f, d)))
    monkeypatch.setenv("GTK_VGPU_ACTIVE", "1")
    assert tr.apply_share_cap({"fractions": [0.25]}, 0, 0) == 0.25 and calls == []
    monkeypatch.delenv("GTK_VGPU_ACTIVE")
    assert tr.apply_share_cap({"fractions": [0.25]}, 0, 0) == 0.25 and calls == [(0.25, 0)]
    assert tr.apply_share_cap({"fractions": [1.0]}, 0, 0) is None


def test_a_new_allocation_never_truncates_a_table_a_live_process_maps(tmp_path):
    """ADVICE r3 (plugin.py:709): each allocation gets fresh config/accounting files.  A process of the
    previous holder that still maps its table (a terminating pod) keeps it intact; the old files are
    removed only once no process holds a slot lock in them."""
    from gpu_topology_on_k8s_amd.deviceplugin import DevicePluginServer, PluginConfig
    from gpu_topology_on_k8s_amd.topology import fixtures as fx
    from gpu_topology_on_k8s_amd.topology.shares import time_slice

    v = time_slice(fx.f7_mi355x(n=2), 4)
    plug = DevicePluginServer(v, PluginConfig(device_specs="stub", dev_root=str(tmp_path), share_guard="env",
                                              guard_dir=str(tmp_path / "g")))
    assert plug.install_guard()

    def acct_of(resp):
        return {m.container_path: m.host_path for m in resp.mounts}[plug.GUARD_ACCT_IN_CONTAINER]

    first = acct_of(plug._container_response([0, 1], {}))
    with open(first, "r+b") as f:
        f.write(b"\x01" * 4096)  # a formatted table
    holder = subprocess.Popen([sys.executable, "-c", "import fcntl, sys\nf = open(sys.argv[1], 'r+b')\n"
                               "fcntl.lockf(f.fileno(), fcntl.LOCK_EX, 1, 16)\nprint('locked', flush=True)\nsys.stdin.readline()",
                               first], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:  # the old pod's process: maps the table and holds a slot lock
        assert holder.stdout.readline().strip() == "locked"
        second = acct_of(plug._container_response([0, 1], {}))
        assert second != first and os.path.exists(first)
        assert open(first, "rb").read(4096) == b"\x01" * 4096  # untouched while it is in use
    finally:
        holder.stdin.write("go\n")
        holder.stdin.flush()
        holder.wait(timeout=30)
    # the old process is gone (its lock with it): the next allocation of those slices removes its files
    third = acct_of(plug._container_response([1], {}))
    assert not os.path.exists(first) and not os.path.exists(first[:-5] + ".conf")
    assert not os.path.exists(second) and os.path.exists(third)  # second was never locked: also collected
    assert os.path.getsize(third) == 0  # fresh; the guard formats it on first use


@pytest.mark.parametrize("fallback", [True, False])
def test_an_address_no_gpu_has_is_reported_and_falls_back(tmp_path, fallback):
    """ADVICE r5 (vgpu_guard.cpp:238): a config address that matches no ROCr agent used to leave the share
    silently unlimited.  Now each such entry is reported on stderr and counted (gtk_vgpu_unmatched, which
    `gtk doctor --gpu` checks); with the fallback ordinal the plugin writes it is applied there, so the
    share still holds."""
    conf = tmp_path / "gtk-vgpu.conf"
    fb = " 0" if fallback else ""
    conf.write_text(f"hbm_limit_bdf 0000:99:00.0 {8 * GiB}{fb}\ncu_mask_bdf 0000:99:00.0 64-127{fb}\n")
    env = {k: v for k, v in os.environ.items() if k not in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES")}
    env.update(GTK_VGPU_CONFIG=str(conf), FAKE_HIP_DEVICE="0")
    env["LD_PRELOAD"] = (env["LD_PRELOAD"] + ":" if env.get("LD_PRELOAD") else "") + str(binary("libgtk_vgpu.so"))
    child = RENUMBER_CHILD.replace('"rocr_ordinal": g.gtk_vgpu_hip_ordinal(0)}',
                                   '"rocr_ordinal": g.gtk_vgpu_hip_ordinal(0), "unmatched": g.gtk_vgpu_unmatched(), '
                                   '"doctor": __import__("gpu_topology_on_k8s_amd.doctor", fromlist=["x"]).check_guard(os.environ)}')
    p = subprocess.run([sys.executable, "-c", child, _fake()], capture_output=True, text=True, timeout=60, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert "0000:99:00.0 matches none of the 2 GPUs" in p.stderr
    assert out["unmatched"] == 2 and out["doctor"][0]["status"] == "fail" and out["doctor"][0]["unmatched"] == 2
    if fallback:
        assert "fallback ROCr ordinal" in p.stderr
        assert out["e"] == [0, 2, 0] and out["total"] == 8 * GiB and out["queue"] == "64-127", out  # still enforced
    else:
        assert "NOT enforced" in p.stderr and out["e"] == [0, 0, 0], out  # loud, not silent


def test_doctor_passes_when_every_address_matched(tmp_path):
    conf = tmp_path / "gtk-vgpu.conf"
    conf.write_text(f"hbm_limit_bdf 0000:05:00.0 {8 * GiB} 0\n")
    env = {k: v for k, v in os.environ.items() if k not in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES")}
    env.update(GTK_VGPU_CONFIG=str(conf), FAKE_HIP_DEVICE="0")
    env["LD_PRELOAD"] = (env["LD_PRELOAD"] + ":" if env.get("LD_PRELOAD") else "") + str(binary("libgtk_vgpu.so"))
    code = ("import ctypes, json, os, sys\nrt = ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_LOCAL)\nn = ctypes.c_int()\n"
            "from gpu_topology_on_k8s_amd.doctor import check_guard\nbefore = check_guard(os.environ)\n"
            "rt.hipGetDeviceCount(ctypes.byref(n))\nprint(json.dumps([before, check_guard(os.environ)]))\n")
    p = subprocess.run([sys.executable, "-c", code, _fake()], capture_output=True, text=True, timeout=60, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    before, after = json.loads(p.stdout.strip().splitlines()[-1])
    assert before[0]["status"] == "skip" and after[0]["status"] == "ok", (before, after)
    assert "matches none" not in p.stderr
