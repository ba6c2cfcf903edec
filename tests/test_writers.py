"""Output formats of src/writer.f90 through the C ABI; CPU only.

Each file is checked byte for byte against the layout the reference writes, and read back
the way the reference's own reader does (tools/read_nrrd_class.py: header lines up to the
first blank line, the data taken from the end of the file; sizes are nz ny nx)."""
import os

import numpy as np
import pytest

from rsmcrt_amd import abi, output, scene
from rsmcrt_amd.engine import SmcrtError


def read_nrrd_like_reference(path):
    """Restatement of read_nrrd_class.read_header/read_data (tools/read_nrrd_class.py:12-99)."""
    types = {"float": np.float32, "double": np.float64}
    with open(path, "rb") as fh:
        lines = iter(fh)
        assert next(lines).decode().startswith("NRRD")
        hdr = {}
        for raw in lines:
            line = raw.decode("ascii", "ignore").rstrip()
            if line == "":
                break
            key, value = line.replace("=", ":").split(":", 1)
            hdr[key.strip()] = value.strip()
        sizes = [int(x) for x in hdr["sizes"].split()]
        dt = np.dtype(types[hdr["type"]])
        n = int(np.prod(sizes))
        fh.seek(-dt.itemsize * n, os.SEEK_END)
        data = np.fromfile(fh, dtype=dt).reshape(sizes)
    return data, hdr


@pytest.mark.parametrize("dtype,name", [(np.float32, "float"), (np.float64, "double")])
def test_nrrd_layout_and_reference_reader(tmp_path, dtype, name):
    rng = np.random.default_rng(1)
    a = rng.random((5, 4, 3)).astype(dtype)  # (nz, ny, nx) = Fortran jmean(3, 4, 5)
    meta = 'nphotons = 1000\nsource = "point"'
    f = output.write_data(tmp_path / "jmean.nrrd", a, metadata=meta)
    blob = open(f, "rb").read()
    head = (f"NRRD0004\ntype: {name}\ndimension: 3\nsizes: 5 4 3\nspace dimension: 3\nencoding: raw\n"
            f"endian: little\n{meta}\n\n\n").encode()
    assert blob == head + a.tobytes()
    data, hdr = read_nrrd_like_reference(f)
    assert hdr["nphotons"] == "1000" and hdr["encoding"] == "raw"
    assert data.dtype == dtype and np.array_equal(data, a)


def test_nrrd_detector_id_and_new_file_names(tmp_path):
    a = np.zeros((2, 2, 2), np.float32)
    p = tmp_path / "escape.nrrd"
    assert output.write_data(p, a, dect_id="det1") == str(p)
    assert b"dector: det1\n" in open(p, "rb").read()
    # get_new_file_name (writer.f90:273-291): existing files are kept unless overwrite
    assert output.write_data(p, a, overwrite=False) == str(tmp_path / "escape (1).nrrd")
    assert output.write_data(p, a, overwrite=False) == str(tmp_path / "escape (2).nrrd")
    assert output.write_data(p, a, overwrite=True) == str(p)


def test_raw_and_unsupported(tmp_path):
    a = np.arange(24, dtype=np.float64).reshape(2, 3, 4)
    f = output.write_data(tmp_path / "j.raw", a)
    assert open(f, "rb").read() == a.tobytes()
    f = output.write_data(tmp_path / "j.dat", a.astype(np.float32))
    assert open(f, "rb").read() == a.astype(np.float32).tobytes()
    with pytest.raises(SmcrtError, match="not supported"):
        output.write_data(tmp_path / "j.txt", a)


def _stream(path):
    return np.fromfile(path, dtype="<f8")


def test_detector_streams(tmp_path):
    circ = scene.circle_dect((0.0, 0.0, 0.5), (0.0, 0.0, 1.0), 1, 0.4, 4)
    data = np.array([1.0, 2.0, 3.0, 4.0, 5.0])
    assert circ.nbins == 5  # TOML nbins + 1 (detectors.f90:132)
    output.write_detector(tmp_path / "d1.dat", circ, data, "ab", 1000)
    s = _stream(tmp_path / "d1.dat")
    head = [1.0, 2.0, ord("a"), ord("b"), 1000.0, 0.4, 0.0, 0.0, 0.5, 0.0, 0.0, 1.0]
    assert np.array_equal(s[:12], head)
    pairs = s[12:].reshape(-1, 2)
    np.testing.assert_array_equal(pairs[:, 0], (np.arange(1, 6) - 0.5) * circ.bin_wid)
    np.testing.assert_array_equal(pairs[:, 1], data)

    ann = scene.annulus_dect((0.0, 0.0, 0.5), (0.0, 0.0, 1.0), 1, 0.1, 0.3, 2)
    output.write_detector(tmp_path / "d3.dat", ann, np.array([7.0, 8.0, 9.0]), "x", 5)
    s = _stream(tmp_path / "d3.dat")
    assert np.array_equal(s[:5], [3.0, 1.0, ord("x"), 5.0, 0.1]) and s[5] == 0.3
    pairs = s[12:].reshape(-1, 2)
    np.testing.assert_array_equal(pairs[:, 0], (np.arange(1, 4) - 0.5) * ann.bin_wid + 0.1)

    cam = scene.camera((-1.0, -1.0, -1.0), (0.0, 2.0, 0.0), (0.0, 0.0, 2.0), 1, 10, 100.0)
    output.write_detector(tmp_path / "d4.dat", cam, np.zeros(121), "cam", 5)
    assert os.path.getsize(tmp_path / "d4.dat") == 0  # not implemented in the reference either


def test_checkpoint(tmp_path):
    g = scene.grid(3, 2, 2, 1.0, 1.0, 1.0)
    j = np.arange(12, dtype=np.float32).reshape(2, 2, 3)
    f = output.write_checkpoint(tmp_path / "ck.dat", "res/scat_test.toml", 12345, j, g)
    assert open(f, "rb").read() == b"tomlfile=res/scat_test.toml\nphotons_run=12345\n" + j.tobytes()


def test_normalise_fluence_matches_fortran_expression():
    g = scene.grid(20, 30, 40, 1.5, 0.75, 2.0)
    j = np.random.default_rng(2).random((40, 30, 20)).astype(np.float32)
    got = output.normalise_fluence(j, g, 123457)
    # writer.f90:46-48, evaluated in fp64 then stored in the fp32 array
    f = (2.0 * 1.5 * 2.0 * 0.75 * 2.0 * 2.0) / (123457 * (2.0 * 1.5 / 20) * (2.0 * 0.75 / 30) * (2.0 * 2.0 / 40))
    assert np.array_equal(got, (j.astype(np.float64) * f).astype(np.float32))
