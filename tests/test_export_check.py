"""The stale dma-buf export checks (ipc.cc ipcAdmitExport) on the CPU: memfd files stand in for the
dma-bufs an export hands back (tests/native/export_check_test.cc). On the GPU the runtime was measured handing one
allocation's export another allocation's dma-buf — of this process or of another one on the same device — which the
zero-copy kernels would then read as if it were the right buffer."""
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_stale_exports_are_refused(built):
    exe = os.path.join(ROOT, "tests", "native", "export_check_test")
    subprocess.check_call(["make", "-s", "tests/native/export_check_test"], cwd=ROOT)
    with tempfile.TemporaryDirectory() as d:
        out = subprocess.run([exe], env=dict(os.environ, NCCL_AMD_DMABUF_NODE_DIR=d), capture_output=True, text=True,
                             timeout=120)
        registry = [f for f in os.listdir(d) if f.endswith(".reg")]
    assert out.returncode == 0, out.stdout + out.stderr
    lines = out.stdout.splitlines()
    assert len(lines) == 8 and all(l.startswith("ok ") for l in lines), out.stdout
    assert registry, "the node registry file was not written in NCCL_AMD_DMABUF_NODE_DIR"
