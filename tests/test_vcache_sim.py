"""CPU replay of the vcache kernel's addressing (spmv-vector-cache_amd/tools/
vc_sim.cpp): every global/LDS index in bounds, no two lanes updating one LDS y
row in the same panel step, ordered geometry bit-exact and split geometry within
the FAST bound -- on the product layout (csrc/plan.cpp) for stripe, ragged,
odd-column and long-row matrices.  Runs without a GPU."""
import os
import subprocess

import hipspmv as hs


def test_vcache_addressing_replay():
    subprocess.run(["make", "-C", hs.PKG_DIR, "lib/vc_sim"], check=True, stdout=subprocess.DEVNULL)
    out = subprocess.run([os.path.join(hs.LIB_DIR, "vc_sim"), "15"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = [l for l in out.stdout.splitlines() if "split=" in l]
    assert sum(": ok" in l for l in lines) >= 16, out.stdout
    assert "VIOLATION" not in out.stderr
    # launch_vcache's guard: the round-1 incident geometry (split-1 kernel, 256 x 8192-row
    # blocks over 2^20 rows) is rejected before any launch, every product layout accepted
    assert "grid guard (incident geometry rejected, product accepted): ok" in out.stdout
    assert "REJECTED" not in out.stdout


def test_layout_builder_and_replay_under_sanitizers():
    # csrc/plan.cpp (the layouts every vcache/wgather launch reads) built with
    # ASan + UBSan, replayed on the scaled stripe, R-MAT and random cases
    subprocess.run(["make", "-C", hs.PKG_DIR, "lib/vc_sim_san"], check=True, stdout=subprocess.DEVNULL)
    out = subprocess.run([os.path.join(hs.LIB_DIR, "vc_sim_san"), "12", "small"], capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert sum(": ok" in l for l in out.stdout.splitlines()) >= 60
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr


def test_vquad_lanes_layout_replay():
    # k_vquad (csrc/vquad.hip) over build_vcache_lanes: every x index inside its panel, every y
    # row inside its block, one owner per row per step, lane pairs and wave-local runs intact,
    # every entry consumed once; u64 exact, f64 within the FAST bound -- plain and under ASan/UBSan
    for tool in ("vq_sim", "vq_sim_san"):
        subprocess.run(["make", "-C", hs.PKG_DIR, f"lib/{tool}"], check=True, stdout=subprocess.DEVNULL)
        out = subprocess.run([os.path.join(hs.LIB_DIR, tool)], capture_output=True, text=True, timeout=900)
        assert out.returncode == 0, out.stdout + out.stderr[-4000:]
        oks = [l for l in out.stdout.splitlines() if l.endswith(": ok")]
        assert any(l.startswith("stripe") for l in oks) and len(oks) >= 8, out.stdout
        assert "VIOLATION" not in out.stderr and "runtime error" not in out.stderr


def test_vflow_layout_replay():
    # k_vflow (csrc/vflow.hip) over build_vflow: every group within its two 64-lane slots, every x
    # index inside its panel slot and every slot element written by the loaders' DMA, every y row
    # updated only by the wave that owns it (the kernel's no-race premise across steps), runs inside
    # a slot, every entry consumed once; u64 exact, f64 within the FAST bound -- plain and under
    # ASan/UBSan (scaled stripe, odd columns, clustered runs, ragged rows, an ineligible shape)
    for tool in ("vf_sim", "vf_sim_san"):
        subprocess.run(["make", "-C", hs.PKG_DIR, f"lib/{tool}"], check=True, stdout=subprocess.DEVNULL)
        out = subprocess.run([os.path.join(hs.LIB_DIR, tool)], capture_output=True, text=True, timeout=900)
        assert out.returncode == 0, out.stdout + out.stderr[-4000:]
        assert "vf_sim: all ok" in out.stdout and sum(l.endswith(": ok") for l in out.stdout.splitlines()) >= 8
        assert "VIOLATION" not in out.stderr and "runtime error" not in out.stderr
