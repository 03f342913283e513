"""Decimal wire strings on the device (fthe_ct_to/from_decimal_dev, fthe_dec.hip):
byte-identical to the host codec (mpz_get_str: the reference's GHEncBatch text,
`stream << g_enc`, distributed_server.cpp:37-54) and to Python's str(int); round
trips; malformed or oversized strings are rejected.  Integer/byte work: exact."""
import numpy as np
import pytest

import pyoracle
from fedtree_amd import _lib
from fedtree_amd.paillier import ct_from_decimal_dev, ct_to_decimal, ct_to_decimal_dev

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from fedtree_amd.paillier import Device
    return Device(0)


def _rows(n, words, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 2**32, (n, words), dtype=np.uint64).astype(np.uint32)
    edge = [np.zeros(words, np.uint32) for _ in range(6)]
    edge[1][0] = 7                                   # one digit
    edge[2][:] = 0xFFFFFFFF                          # the longest string
    edge[3][:words // 2] = a[0, :words // 2] if n else 5   # leading zero words
    edge[4][0] = 999999999                           # exactly one full chunk
    edge[5][0], edge[5][1] = 1000000000 % 2**32, 0   # 10^9: a chunk boundary
    return np.concatenate([np.stack(edge), a])


@pytest.mark.parametrize("words,n", [(128, 4000), (64, 777), (32, 300), (127, 50)])
def test_decimal_dev_matches_host_and_python(dev, words, n):
    import torch
    a = _rows(n, words, words + n)
    ct = torch.from_numpy(a.view(np.int32)).to("cuda:0")
    buf, offs = ct_to_decimal_dev(dev, ct)
    dev.sync()
    o = offs.cpu().numpy()
    raw = buf[: int(o[-1])].cpu().numpy().tobytes()
    got = [raw[o[i]:o[i + 1]].decode() for i in range(len(a))]
    assert got == ct_to_decimal(a)                                 # the host (GMP) codec
    assert got[:64] == [str(v) for v in pyoracle.words_to_ints(a[:64])]
    back = ct_from_decimal_dev(dev, buf, offs, words)
    dev.sync()
    assert np.array_equal(back.cpu().numpy().view(np.uint32), a)


def test_decimal_dev_full_size_roundtrip(dev):
    """1M P-2048 ciphertext-sized rows (128 words): device round trip, host spot checks."""
    import torch
    g = torch.Generator(device="cuda:0").manual_seed(3)
    ct = torch.randint(-2**31, 2**31 - 1, (1 << 20, 128), dtype=torch.int32, device="cuda:0", generator=g)
    buf, offs = ct_to_decimal_dev(dev, ct)
    back = ct_from_decimal_dev(dev, buf, offs, 128)
    dev.sync()
    assert torch.equal(back, ct)
    idx = np.arange(0, 1 << 20, 65537)
    o = offs.cpu().numpy()
    raw = buf[: int(o[-1])].cpu().numpy().tobytes()
    rows = ct[torch.from_numpy(idx).to("cuda:0")].cpu().numpy().view(np.uint32)
    assert [raw[o[i]:o[i + 1]].decode() for i in idx] == ct_to_decimal(rows)


def test_decimal_dev_errors(dev):
    import torch
    words = 4

    def parse(strings):
        enc = [s.encode() for s in strings]
        offs = torch.tensor(np.concatenate([[0], np.cumsum([len(x) for x in enc])]), dtype=torch.int64,
                            device="cuda:0")
        buf = torch.tensor(np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8).copy(), device="cuda:0")
        return ct_from_decimal_dev(dev, buf, offs, words)

    ok = parse(["0", "123", str(2**128 - 1)])
    assert pyoracle.words_to_ints(ok.cpu().numpy().view(np.uint32)) == [0, 123, 2**128 - 1]
    for bad in (["12a"], [""], [str(2**128)], ["1" * 60], ["-5"]):
        with pytest.raises(_lib.FtheError):
            parse(bad)
    # output buffer too small: FTHE_ERR_ARG and offsets[count] = bytes needed
    ct = torch.full((3, words), -1, dtype=torch.int32, device="cuda:0")
    buf = torch.empty(10, dtype=torch.uint8, device="cuda:0")
    offs = torch.empty(4, dtype=torch.int64, device="cuda:0")
    import ctypes
    dev.order_in()                   # direct C-ABI call: after torch's fill of ct
    rc = dev.lib.fthe_ct_to_decimal_dev(dev.ctx, ctypes.c_void_p(ct.data_ptr()), words, 3,
                                        ctypes.c_void_p(buf.data_ptr()), 10, ctypes.c_void_p(offs.data_ptr()))
    assert rc == _lib.FTHE_ERR_ARG and int(offs[-1]) == 3 * len(str(2**128 - 1))
