import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def load_golden(name):
    """Fixtures are plain arrays: np.load with allow_pickle=False (the default)."""
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def golden():
    return load_golden


def cases(z, suffix):
    return sorted({k.split("/")[0] for k in z.files if k.endswith("/" + suffix)})


def assert_ref_parity(got, ref32, ref64, rtol=1e-3, afrac=1e-4, frac_ok=0.95):
    """Parity with a reference fp32 output whose own rounding noise is known (ref64 = the same
    reference module run in fp64).  Two checks:
      * conditioning: max |got - ref64| <= 2 max |ref32 - ref64| + afrac * scale -- ``got`` is at
        least as close to the exact answer as the reference's own fp32 result, up to 2x;
      * element-wise: |got - ref32| <= rtol |ref32| + afrac * scale for >= frac_ok of the elements
        (the rest sit downstream of a gate within ~1e-5 of 0, where x / sqrt(x^2 + 1e-6) amplifies any
        rounding ~1e3x; one such gate moves all V logits of its frame, so on the tiny
        fixtures a single flipped gate is several % of the elements).
    scale = max(1, max |ref32|)."""
    got = np.asarray(got, np.float64)
    ref32 = np.asarray(ref32, np.float64)
    ref64 = np.asarray(ref64, np.float64)
    scale = max(1.0, float(np.abs(ref32).max()))
    noise = float(np.abs(ref32 - ref64).max())
    err64 = float(np.abs(got - ref64).max())
    assert err64 <= 2 * noise + afrac * scale, (err64, noise)
    ok = np.abs(got - ref32) <= rtol * np.abs(ref32) + afrac * scale
    assert ok.mean() >= frac_ok, (ok.mean(), float(np.abs(got - ref32).max()))
    return err64, noise, float(ok.mean())
