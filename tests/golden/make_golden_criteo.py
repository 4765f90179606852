"""Golden fixtures for the Criteo input path (§8(f) #4), produced by running PyTorch on the
reference's own transform (data_loader_terabyte.py @ 2024-10-24):

  CriteoBinDataset.__getitem__ (:227-237): tensor = from_numpy(int32 records).view(-1, 40);
  _transform_features(x_int=tensor[:, 1:14], x_cat=tensor[:, 14:], y=tensor[:, 0],
                      max_ind_range, flag_input_torch_tensor=True)              (:68-87)

restated op for op with torch (the reference module itself cannot be imported here).
Records include negative / huge dense values (log of 0 and of negatives), int32 extremes,
negative categoricals under the modulo, and a batch that is not a multiple of 64.
Run: python tests/golden/make_golden_criteo.py   (writes tests/golden/criteo.npz)"""
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def transform_features(x_int_batch, x_cat_batch, y_batch, max_ind_range):  # :68-87, tensor branch
    if max_ind_range > 0:
        x_cat_batch = x_cat_batch % max_ind_range
    x_int_batch = torch.log(x_int_batch.clone().detach().type(torch.float) + 1)
    x_cat_batch = x_cat_batch.clone().detach().type(torch.long)
    y_batch = y_batch.clone().detach().type(torch.float32).view(-1, 1)
    batch_size = x_cat_batch.shape[0]
    feature_count = x_cat_batch.shape[1]
    lS_o = torch.arange(batch_size).reshape(1, -1).repeat(feature_count, 1)
    return x_int_batch, lS_o, x_cat_batch.t(), y_batch.view(-1, 1)


def records(B, seed):
    rs = np.random.RandomState(seed)
    rec = np.zeros((B, 40), np.int64)
    rec[:, 0] = rs.randint(0, 2, B)
    rec[:, 1:14] = np.floor(np.exp(rs.uniform(0, 10, (B, 13))) - 1).astype(np.int64)
    rec[:, 14:] = rs.randint(0, 2 ** 31 - 1, (B, 26))
    rec[0, 1:14] = [-1, -2, 0, 1, 2 ** 24 + 1, 2 ** 31 - 1, -(2 ** 31), 16777217, 3, 7, 1000000, 65535, 12]
    rec[1, 14:] = [-1, -(2 ** 31), 2 ** 31 - 1, 0, 9999999, 10000000, 10000001, -10000001] + [5] * 18
    return rec.astype(np.int32)


def main():
    out = {}
    for name, B, seed, mod in (("a", 300, 11, 10_000_000), ("b", 2048, 12, -1), ("c", 64, 13, 97)):
        rec = records(B, seed)
        t = torch.from_numpy(rec).view((-1, 40))
        X, lS_o, lS_i, y = transform_features(t[:, 1:14], t[:, 14:], t[:, 0], mod)
        out.update({f"{name}_rec": rec, f"{name}_mod": np.int64(mod), f"{name}_X": X.numpy(),
                    f"{name}_lS_o": lS_o.numpy(), f"{name}_lS_i": lS_i.contiguous().numpy(), f"{name}_y": y.numpy()})
    out["torch_version"] = np.array(torch.__version__)
    np.savez_compressed(os.path.join(HERE, "criteo.npz"), **out)
    print("wrote criteo.npz", torch.__version__)


if __name__ == "__main__":
    main()
