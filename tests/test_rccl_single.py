"""The RCCL branch of TorchComm (hbmr/parallel/collectives.py) on a real
process group: one GPU allows only a 1-rank ``nccl`` group (RCCL refuses two
ranks on one device), but that still runs RCCL's communicator set-up on the
MI355X and every device-to-device collective the data plane uses — the
K-Means all-reduce of int64 partials, the TeraSort / WordCount all-to-all-v,
all-gather, broadcast, reduce-scatter — instead of the gloo-staged path the
multi-rank rehearsal takes.  Run in a child process so the test session keeps
no process group."""
import os
import subprocess
import sys
import textwrap

import pytest

_SCRIPT = textwrap.dedent(r"""
    import datetime, os, sys
    sys.path.insert(0, os.environ["HBMR_ROOT"])
    import torch
    import torch.distributed as dist
    from hbmr.parallel.collectives import TorchComm
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="file://" + sys.argv[1], rank=0, world_size=1,
                            timeout=datetime.timedelta(seconds=60), device_id=dev)
    comm = TorchComm(group=None, cpu_group=dist.new_group(backend="gloo"))
    assert comm.backend == "nccl" and not comm.stage, comm.backend
    x = torch.arange(1 << 20, dtype=torch.int64, device=dev) * 3
    ref = x.clone()
    comm.all_reduce(x)
    assert torch.equal(x, ref)
    f = torch.randn(4096, 128, device=dev)
    g = comm.all_gather(f)
    assert len(g) == 1 and torch.equal(g[0], f)
    send = torch.randint(0, 255, (1 << 20,), dtype=torch.uint8, device=dev)
    recv, rcounts = comm.all_to_all_v(send, [send.numel()])
    assert rcounts == [send.numel()] and torch.equal(recv, send) and recv.is_cuda
    outs = comm.all_to_all([torch.ones(7, 3, device=dev)])
    assert len(outs) == 1 and outs[0].shape == (7, 3) and outs[0].is_cuda
    b = torch.full((1000,), 5.0, device=dev)
    comm.broadcast(b, 0)
    assert torch.all(b == 5.0)
    rs = comm.reduce_scatter(torch.ones(10, 4, device=dev))
    assert rs.shape == (10, 4) and torch.all(rs == 1.0)
    h = torch.arange(10, dtype=torch.int64)            # host tensor: the gloo group
    comm.all_reduce(h)
    assert torch.equal(h, torch.arange(10, dtype=torch.int64))
    comm.barrier()
    torch.cuda.synchronize()
    assert sum(v for k, v in comm.stats.items() if k.endswith("_STAGED")) == 0, dict(comm.stats)
    dist.destroy_process_group()
    print("RCCL_OK", flush=True)
""")


@pytest.mark.gpu
def test_torchcomm_rccl_branch_on_one_gpu(tmp_path):
    env = dict(os.environ, HBMR_ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-c", _SCRIPT, str(tmp_path / "pg")], env=env,
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0 and "RCCL_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
