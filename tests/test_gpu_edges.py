"""Edge cases on the GPU (gpu): empty inputs, a bucket past 2^31 bytes (64-bit
indexing), the single-message allreduce_write (the reference posts a 2-message
window unconditionally, api.c:408, and would read past src), zero-length calls."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_empty_inputs(gpu):
    import torch
    from container_inc_amd import inccl
    e = torch.empty(0, device=gpu)
    assert inccl.quantise(e, 25).numel() == 0
    assert inccl.reduce_f32([e, e], 25).numel() == 0
    assert inccl.sum_q32([torch.empty(0, dtype=torch.int32, device=gpu)] * 3).numel() == 0
    assert inccl.checksum_q32(torch.empty(0, dtype=torch.int32, device=gpu)) == 0
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    assert comm.allreduce_f32([e], scale_exp=25).numel() == 0
    dst = np.full(10, 5, np.int32)
    comm.allreduce_write(np.zeros(10, np.int32), 0, dst)       # len 0: nothing reduced
    comm.allreduce_write(np.zeros(10, np.int32), 10, dst)      # < one message: nothing reduced (api.c:406)
    assert np.all(dst == 5)
    comm.destroy()
    grp.destroy()


def test_single_message_len(gpu, orc):
    """len = 1024: one whole message; the reference's window would read a second
    message past src (api.c:408) -- here exactly one message is reduced."""
    import threading
    from container_inc_amd import inccl
    xs = [np.arange(1024, dtype=np.int32) * (r + 1) for r in range(2)]
    outs = [None, None]

    def rank(r):
        g = inccl.inccl_group_create_local(2, r, "single-msg")
        c = inccl.inccl_communicator_create(g, 4096)
        d = np.zeros(1024, np.int32)
        c.allreduce_write(xs[r], 1024, d)
        outs[r] = d
        c.destroy()
        g.destroy()

    th = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    for d in outs:
        np.testing.assert_array_equal(d, 3 * np.arange(1024, dtype=np.int32))


def test_bucket_past_2gib(gpu, orc):
    """n = 2^29 + 3 fp32 elements (2 GiB + 12 B): 64-bit offsets in every kernel."""
    import torch
    from container_inc_amd import inccl
    n = (1 << 29) + 3
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(n, generator=g)
    xd = x.to(gpu)
    out = inccl.reduce_f32([xd], 20)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    want = orc.reduce_f32([x.numpy()], 20)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    q = inccl.quantise(xd, 20)
    assert inccl.checksum_q32(q) == orc.checksum_q32(orc.quantise(x.numpy(), 20))
