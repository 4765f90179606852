"""GPU: the Criteo input path through dqrm_criteo_unpack against the
torch fixture of _transform_features (data_loader_terabyte.py:68-87): integer outputs
bit-exact, log(x+1) within 2 ulp (device logf vs torch's CPU log) with identical NaN/-inf
positions; CriteoBinDataset / CriteoPrefetcher over a binary file; and the unpacked
[26, B] indices driving the embedding forward directly."""
import os

import numpy as np
import pytest
import torch

import gen_inputs as G
import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def CR():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import deep_quantized_recommendation_model_dqrm_amd as d

    d._lib.load()
    from deep_quantized_recommendation_model_dqrm_amd import criteo

    return criteo


def ulp_diff(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    same = (np.isnan(a) & np.isnan(b)) | (np.isinf(a) & (a == b))
    d = np.abs(a.view(np.int32).astype(np.int64) - b.view(np.int32).astype(np.int64))
    d[same] = 0
    return d


@pytest.mark.parametrize("case", ["a", "b", "c"])
def test_unpack_matches_torch_fixture(CR, golden_dir, case):
    fx = dict(np.load(os.path.join(golden_dir, "criteo.npz")))
    rec = torch.from_numpy(fx[f"{case}_rec"]).cuda()
    X, lS_o, lS_i, y = CR.transform_features(rec, int(fx[f"{case}_mod"]))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(lS_i.cpu().numpy(), fx[f"{case}_lS_i"])
    np.testing.assert_array_equal(lS_o.cpu().numpy(), fx[f"{case}_lS_o"])
    np.testing.assert_array_equal(y.cpu().numpy(), fx[f"{case}_y"])
    Xg = X.cpu().numpy()
    assert ulp_diff(Xg, fx[f"{case}_X"]).max() <= 2
    assert np.array_equal(np.isnan(Xg), np.isnan(fx[f"{case}_X"]))


def test_unpack_sizes_and_no_offsets(CR):
    for B in (1, 63, 64, 65, 4097, 600_000):  # > 8192 workgroups: grid-stride passes
        rs = np.random.RandomState(B)
        rec = rs.randint(-5, 1 << 30, (B, 40)).astype(np.int32)
        X, lS_o, lS_i, y = CR.transform_features(torch.from_numpy(rec).cuda(), 1 << 20, with_offsets=False)
        assert lS_o is None
        Xo, _, lS_io, yo = O.criteo_transform(rec, 1 << 20)
        np.testing.assert_array_equal(lS_i.cpu().numpy(), lS_io)
        np.testing.assert_array_equal(y.cpu().numpy(), yo)
        assert ulp_diff(X.cpu().numpy(), Xo).max() <= 2
    X, lS_o, lS_i, y = CR.transform_features(torch.zeros(0, 40, dtype=torch.int32, device="cuda"))
    assert X.shape == (0, 13) and lS_i.shape == (26, 0)


def test_dataset_prefetcher_and_forward(CR, tmp_path):
    import deep_quantized_recommendation_model_dqrm_amd as dq

    rows = [min(n, 5000) for n in G.KAGGLE_ROWS]
    rs = np.random.RandomState(3)
    n = 700
    y = rs.randint(0, 2, n)
    xi = rs.randint(0, 1000, (n, 13))
    xc = rs.randint(0, 1 << 30, (n, 26))
    f = str(tmp_path / "day.bin")
    CR.numpy_to_binary([(y, xi, xc)], f)
    ds = CR.CriteoBinDataset(f, batch_size=256, max_ind_range=5000, device="cuda")
    assert len(ds) == 3
    ts = dq.EmbeddingTableSet([5000] * 26, 16, device="cuda", init="uniform", seed=9)
    got = list(CR.CriteoPrefetcher(ds))
    assert len(got) == 3
    for k, (X, lS_o, lS_i, yb) in enumerate(got):
        ref = O.criteo_transform(ds.records(k), 5000)
        np.testing.assert_array_equal(lS_i.cpu().numpy(), ref[2])
        np.testing.assert_array_equal(yb.cpu().numpy(), ref[3])
        direct = ds[k]
        assert torch.equal(direct[2], lS_i) and torch.equal(direct[1], lS_o)
        # the unpacked indices feed the QAT forward as a Criteo-form batch
        y1 = ts.forward(ds.lookup_batch(lS_i))
        y2 = ts.forward(dq.LookupBatch(torch.from_numpy(ref[2]).cuda(), torch.from_numpy(ref[1]).cuda()))
        assert torch.equal(y1, y2)
    assert ts.read_errors() == 0


def test_collate_wrapper(CR):
    rs = np.random.RandomState(4)
    tuples = [(rs.randint(0, 50, 13), rs.randint(0, 10 ** 7, 26), rs.randint(0, 2)) for _ in range(128)]
    X, lS_o, lS_i, T = CR.collate_wrapper_criteo_offset(tuples)
    rec = np.array([[t[2], *t[0], *t[1]] for t in tuples], np.int32)
    Xo, lS_oo, lS_io, To = O.criteo_transform(rec, -1)
    np.testing.assert_array_equal(lS_i.cpu().numpy(), lS_io)
    np.testing.assert_array_equal(lS_o.cpu().numpy(), lS_oo)
    np.testing.assert_array_equal(T.cpu().numpy(), To)
    assert ulp_diff(X.cpu().numpy(), Xo).max() <= 2
