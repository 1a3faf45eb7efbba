"""PLY IO of Gaussian models.  CPU part: the host header /
row codec against the oracle's restatement of the bytes plyfile writes for the
reference's save_ply (parity unpinned against plyfile itself, which is absent);
GPU part: save_ply / load_ply / merge_ply through the arena transposition kernels."""
import os

import numpy as np
import pytest
import torch

from oracle import train_oracle as TO


def _matrix(P, M, C=2, seed=0):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g)
    raw = {"xyz": r(P, 3), "f_dc": r(P, 1, 3), "f_rest": r(P, M - 1, 3), "opacity": r(P, 1), "segment": r(P, C),
           "scaling": r(P, 3), "rotation": r(P, 4)}
    return raw, TO.ply_attribute_matrix(raw["xyz"], raw["f_dc"], raw["f_rest"], raw["opacity"], raw["segment"],
                                        raw["scaling"], raw["rotation"])


def test_attribute_names_match_reference_order():
    from gsr_train import ply
    n = ply.attribute_names(16, 2)
    assert n[:9] == ["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"]
    assert n[9] == "f_rest_0" and n[9 + 44] == "f_rest_44" and n[54] == "opacity"
    assert n[55:] == ["segment_0", "segment_1", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3"]
    assert len(n) == 6 + 48 + 1 + 2 + 3 + 4


def test_writer_bytes_equal_reference_layout(tmp_path):
    from gsr_train import ply
    names = ply.attribute_names(16, 2)
    _, mat = _matrix(37, 16)
    p = tmp_path / "a.ply"
    ply.write_rows(str(p), names, mat)
    assert p.read_bytes() == TO.ply_reference_bytes(names, mat)


@pytest.mark.parametrize("fmt,ptype", [("binary_little_endian", "float"), ("binary_big_endian", "float"),
                                       ("binary_little_endian", "double"), ("ascii", "float")])
def test_reader_formats(tmp_path, fmt, ptype):
    from gsr_train import ply
    names = ply.attribute_names(4, 2)
    _, mat = _matrix(23, 4, seed=1)
    p = tmp_path / "b.ply"
    p.write_bytes(TO.ply_reference_bytes(names, mat, fmt=fmt, prop_type=ptype))
    got_names, rows = ply.read_rows(str(p))
    assert got_names == names and rows.dtype == np.float32
    np.testing.assert_array_equal(rows, mat)


def test_column_map_is_the_reference_transpose():
    """arena float (coefficient m, channel c) <- f_dc_c (m = 0) or f_rest_{c(M-1)+m-1}."""
    from gsr_train import ply
    M = 16
    names = ply.attribute_names(M, 2)
    col = ply.arena_columns(names, M, 2)
    raw, mat = _matrix(5, M)
    feats = torch.cat([raw["f_dc"], raw["f_rest"]], dim=1).numpy()  # [P, M, 3] = arena order
    arena_rows = mat[:, col]
    np.testing.assert_array_equal(arena_rows[:, 3:3 + 3 * M].reshape(5, M, 3), feats)
    np.testing.assert_array_equal(arena_rows[:, 3 + 3 * M + 1:3 + 3 * M + 4], raw["scaling"].numpy())
    with pytest.raises(ValueError):
        ply.arena_columns(names, 9, 2)  # f_rest count mismatch (gaussian_model.py:283 assert)
    with pytest.raises(KeyError):
        ply.arena_columns([n for n in names if n != "rot_2"], M, 2)


@pytest.mark.gpu
def test_save_load_merge_roundtrip_gpu(tmp_path, gpu_available):
    from gsr_train import GaussianModel, ply
    raw, mat = _matrix(3001, 16, seed=3)
    m = GaussianModel(3, device="cuda")
    m.create_from_tensors(raw["xyz"], raw["f_dc"], raw["f_rest"], raw["opacity"], raw["segment"], raw["scaling"],
                          raw["rotation"])
    p = tmp_path / "pc" / "point_cloud.ply"
    m.save_ply(str(p))
    assert p.read_bytes() == TO.ply_reference_bytes(ply.attribute_names(16, 2), mat)
    m2 = GaussianModel(3, device="cuda")
    m2.load_ply(str(p))
    assert m2.active_sh_degree == 3 and m2.num_points == 3001
    assert torch.equal(m2._arena.data[:m2._spec.off[6]].cpu(), m._arena.data.cpu())
    # host arrays of load_ply_no_instance + instance_parm give the same model
    arrs = m2.load_ply_no_instance(str(p))
    m3 = GaussianModel(3, device="cuda")
    m3.instance_parm(*arrs)
    assert torch.equal(m3._arena.data.cpu(), m._arena.data.cpu())
    # merge: two scenes concatenated in order with per-scene offsets
    raw2, mat2 = _matrix(1500, 16, seed=4)
    q = tmp_path / "second.ply"
    q.write_bytes(TO.ply_reference_bytes(ply.attribute_names(16, 2), mat2))
    m4 = GaussianModel(3, device="cuda")
    offsets, ids = m4.merge_ply([str(p), str(q)])
    assert offsets == [(0, 3001), (3001, 4501)]
    assert int(ids[3000]) == 0 and int(ids[3001]) == 1
    both = np.concatenate([mat, mat2])
    rows = ply.arena_to_rows(m4._spec, m4._arena.data, ply.attribute_names(16, 2)).cpu().numpy()
    np.testing.assert_array_equal(rows, both)
    # save with a mask writes the selected rows only
    mask = torch.arange(4501, device="cuda") % 3 == 0
    m4.save_ply_using_mask(str(tmp_path / "masked.ply"), mask)
    _, mrows = ply.read_rows(str(tmp_path / "masked.ply"))
    np.testing.assert_array_equal(mrows, both[mask.cpu().numpy()])
