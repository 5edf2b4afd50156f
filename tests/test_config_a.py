"""BASELINE config A — the reference's CPU-runnable case: 2-input fp32
ncclSum over a 4 MiB bucket (1,048,576 elements per input), world_size = 1,
inputs uniform[-1, 1) seeded 1234 + source index.

CPU: the oracle's fold equals an independent numpy float32 left fold bitwise
(the plumbing check, no GPU). GPU: the reduction core (device-resident), the
host-staged entry point (sources and result in host memory, the emulator's
proxy/net buffers) and ncclAllReduce / ncclReduce at world_size = 1 all match
the oracle bitwise."""
import numpy as np
import pytest

COUNT = 1 << 20


def _inputs(oracle):
    return oracle.random_inputs(7, 2, COUNT, seed=1234)


def test_config_a_cpu_oracle(oracle):
    a, b = _inputs(oracle)
    assert a.dtype == np.float32 and a.size == COUNT
    got = oracle.reduce_multi([a, b], 7, 0)[0]
    assert np.array_equal(got.view(np.uint32), (a + b).view(np.uint32))


@pytest.mark.gpu
def test_config_a_gpu(nbx, oracle, torch_gpu):
    torch = torch_gpu
    a, b = _inputs(oracle)
    exp = oracle.reduce_multi([a, b], 7, 0)[0].view(np.uint32)
    st = torch.cuda.current_stream().cuda_stream
    op = nbx.host_to_dev_redop(nbx.ncclRedOp.ncclSum, nbx.ncclDataType.ncclFloat32, 1)
    ta, tb = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    out = torch.empty_like(ta)
    nbx.reduce_multi([out.data_ptr()], [ta.data_ptr(), tb.data_ptr()], COUNT, 7, op, 0, False, st)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), exp)
    # host-staged: pinned host sources and destination
    ha, hb = torch.from_numpy(a).pin_memory(), torch.from_numpy(b).pin_memory()
    ho = torch.empty_like(ha).pin_memory()
    nbx.reduce_multi_host([ho.data_ptr()], [ha.data_ptr(), hb.data_ptr()], COUNT, 7, op, 0, False, st)
    assert np.array_equal(ho.numpy().view(np.uint32), exp)
    # world_size = 1 through the NCCL API: AllReduce / Reduce of one rank are copies (onerank.cu:50-55)
    comm = nbx.Communicator.init_rank(1, nbx.get_unique_id(), 0)
    y = torch.empty_like(ta)
    comm.all_reduce(out.data_ptr(), y.data_ptr(), COUNT, 7, 0, st)
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy().view(np.uint32), exp)
    y.zero_()
    comm.reduce(out.data_ptr(), y.data_ptr(), COUNT, 7, 0, 0, st)
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy().view(np.uint32), exp)
    comm.destroy()
