"""Issue-order model of the explicit vmcnt waits in the asm-loaded rings
(csrc/vcache.hip CX == 2 / LD == 2, csrc/wgather.hip k_wgather_pipe).

On gfx9 vector-memory loads retire in issue order, so `s_waitcnt vmcnt(N)`
guarantees every load except the N youngest has landed.  Each model below
replays one wave's sequence of loads and waits as the kernel issues them
(prologue, peeled first step, the padded DE-unrolled steps) and checks that
every register-ring value is consumed only after a wait that retired its
load; a wait stronger than necessary costs time, not correctness, so only
the safety direction is asserted.  The last test runs tools/vmcnt_check.py
(a dataflow check over the compiled kernels' control-flow graphs) on every
k_vcache and gather instantiation.  Test infrastructure, CPU only."""
import pytest


class Wave:
    def __init__(self):
        self.issued = []  # load ids in issue order
        self.landed = set()

    def load(self, tag):
        self.issued.append(tag)

    def wait(self, n):  # vmcnt(n): all but the n youngest have landed
        pending = [t for t in self.issued if t not in self.landed]
        for t in pending[:max(0, len(pending) - n)]:
            self.landed.add(t)

    def use(self, tag):
        assert tag in self.landed, f"{tag} consumed before its load retired"


def vcache_compute_ring(npu, DE, EPT):
    """k_vcache compute role, CX == 2: load_e(s) issues 2*EPT loads; every
    step of the padded loop waits vmcnt((DE-1)*2*EPT), consumes slot s (a
    real step only), issues load_e(s+DE)."""
    w = Wave()
    for s in range(DE):
        for j in range(2 * EPT):
            w.load(("e", s, j))
    align = DE if DE % 2 == 0 else 2 * DE
    for s in range((npu + align - 1) // align * align):
        w.wait((DE - 1) * 2 * EPT)
        if s < npu:
            for j in range(2 * EPT):
                w.use(("e", s, j))
        for j in range(2 * EPT):
            w.load(("e", s + DE, j))
    w.wait(0)


def vcache_loader_ring(npu, NJ):
    """k_vcache loader role, LD == 2: load x0, wait 0, store x0, load x1, x2;
    step s waits vmcnt(NJ), stores x(s+1), loads x(s+3)."""
    w = Wave()
    for j in range(NJ):
        w.load(("x", 0, j))
    w.wait(0)
    for j in range(NJ):
        w.use(("x", 0, j))
    for p in (1, 2):
        for j in range(NJ):
            w.load(("x", p, j))
    for s in range((npu + 3) // 4 * 4):  # padded like the compute role (DE = 4)
        w.wait(NJ)
        if s + 1 < npu:
            for j in range(NJ):
                w.use(("x", s + 1, j))
        for j in range(NJ):
            w.load(("x", s + 3, j))
    w.wait(0)


def wgather_pipe(npanels, DE, EPT):
    """k_wgather_pipe: E(0..DE-1), wait 0, G(0); step 0 peeled: G(1), wait EPT,
    consume, E(DE); steps 1 .. nsteps-1 (padded to whole groups of DE): wait
    (DE-2)*3*EPT, G(s+1) [needs E(s+1)], wait 3*EPT, consume E(s), G(s),
    issue E(s+DE)."""
    w = Wave()
    for s in range(DE):
        for j in range(2 * EPT):
            w.load(("e", s, j))
    w.wait(0)
    for j in range(2 * EPT):
        w.use(("e", 0, j))  # gather(0) reads the codes of step 0
    for j in range(EPT):
        w.load(("g", 0, j))
    for j in range(2 * EPT):
        w.use(("e", 1, j))  # gather(1) in the peeled step
    for j in range(EPT):
        w.load(("g", 1, j))
    w.wait(EPT)
    for j in range(EPT):
        w.use(("g", 0, j))
    for j in range(2 * EPT):
        w.load(("e", DE, j))
    nsteps = 1 + (npanels - 1 + DE - 1) // DE * DE
    for s in range(1, nsteps):
        w.wait((DE - 2) * 3 * EPT)
        for j in range(2 * EPT):
            w.use(("e", s + 1, j))  # gather(s+1) reads the codes of step s+1
        for j in range(EPT):
            w.load(("g", s + 1, j))
        w.wait(3 * EPT)
        for j in range(EPT):
            w.use(("g", s, j))
        for j in range(2 * EPT):
            w.use(("e", s, j))
        for j in range(2 * EPT):
            w.load(("e", s + DE, j))
    w.wait(0)


@pytest.mark.parametrize("npu", [1, 2, 3, 4, 5, 7, 8, 87, 133])
@pytest.mark.parametrize("DE,EPT", [(4, 3), (4, 2), (2, 3), (6, 2)])
def test_vcache_compute_ring_waits(npu, DE, EPT):
    vcache_compute_ring(npu, DE, EPT)


@pytest.mark.parametrize("npu", [1, 2, 3, 4, 87, 130])
@pytest.mark.parametrize("NJ", [8, 4, 1])
def test_vcache_loader_ring_waits(npu, NJ):
    vcache_loader_ring(npu, NJ)


@pytest.mark.parametrize("npanels", [1, 2, 3, 4, 5, 8, 128])
@pytest.mark.parametrize("DE,EPT", [(4, 2), (4, 4), (2, 2), (6, 3)])
def test_wgather_pipe_waits(npanels, DE, EPT):
    wgather_pipe(npanels, DE, EPT)


def test_model_catches_a_short_wait():
    # the model must reject a wait that leaves the consumed load in flight
    w = Wave()
    w.load("a")
    w.load("b")
    w.wait(2)
    with pytest.raises(AssertionError):
        w.use("a")


def test_compiled_rings_pass_the_dataflow_check(tmp_path):
    """tools/vmcnt_check.py on the compiled kernels, product and experimental
    builds: every instantiation of k_vcache, of the gather kernels (k_wgather,
    k_wgather_split, k_wgather_pipe), of k_sell / k_sell_iso and of k_vquad
    (asm x and entry rings, csrc/vquad.hip) reads no
    VGPR a vector-memory load may still be writing, and copies none (a copy of
    an in-flight ring register at a loop edge was the round-4 probe's fault)."""
    import os
    import subprocess
    import sys
    import hipspmv as hs
    csrc = os.path.join(hs.PKG_DIR, "csrc")
    # the product build, and the experimental build (make EXPERIMENTAL=1) with every instantiation
    least = {("vcache.hip", 0): 14, ("vcache.hip", 1): 46, ("wgather.hip", 0): 26, ("wgather.hip", 1): 26,
             ("sell.hip", 0): 6, ("sell.hip", 1): 6, ("vquad.hip", 1): 54}
    for (src, exp), n in least.items():
        asm = tmp_path / f"{src}.{exp}.s"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        f"-I{os.path.join(hs.REPO_DIR, 'include')}", f"-I{csrc}", "--cuda-device-only", "-S",
                        *(["-DHIPSPMV_EXPERIMENTAL_KERNELS"] if exp else []),
                        os.path.join(csrc, src), "-o", str(asm)], check=True, capture_output=True)
        out = subprocess.run([sys.executable, os.path.join(hs.PKG_DIR, "tools", "vmcnt_check.py"), str(asm)],
                             capture_output=True, text=True)
        assert out.returncode == 0, out.stdout
        assert out.stdout.count(": 0 violations") >= n, (src, exp, out.stdout)


def test_overlap_probe_rings_pass_the_dataflow_check(tmp_path):
    """The round-4 overlap probe's GPU fault (DESIGN.md
    §9.4): its k_gather (the G skeletons) read and overwrote VGPRs that asm
    loads were still writing -- 35 violations in the D=0 instantiation of the
    faulting revision (13a60ea), among them an address register rewritten under
    an in-flight load -- and the fault surfaced at the synchronisation after
    G's warm-up launches (overlap_probe.hip:306 there).  The fixed probe ties
    every asm-loaded register to its wait (vm_wait_tie): every kernel in it
    passes tools/vmcnt_check.py."""
    import os
    import subprocess
    import sys
    import hipspmv as hs
    src = os.path.join(hs.PKG_DIR, "tools", "overlap_probe.hip")
    asm = tmp_path / "overlap_probe.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "--cuda-device-only", "-S", src, "-o", str(asm)], check=True, capture_output=True)
    out = subprocess.run([sys.executable, os.path.join(hs.PKG_DIR, "tools", "vmcnt_check.py"), str(asm)],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    lines = [l for l in out.stdout.splitlines() if "violations" in l]
    assert len(lines) >= 20 and all(l.endswith(": 0 violations") for l in lines), out.stdout
    assert any("k_gather" in l for l in lines)
