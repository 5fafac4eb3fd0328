"""GPU-build getters of the extractor (orbfe_extractor_levels / orbfe_extractor_scale_info) against
the known answers SURVEY.md §8 derives from the reference source and against the oracle.

These are the tables ORBextractor exposes through GetLevels / GetScaleFactors /
GetInverseScaleFactors / GetScaleSigmaSquares / GetInverseScaleSigmaSquares (ORBextractor.h:61-81,
ORBextractor.cc:409-445) and Frame copies into every frame (Frame.cc:110-116); the C++ shim copies
them straight from orbfe_extractor_scale_info (shim/ORBextractor_orbfe.cc)."""
import numpy as np
import pytest

from test_tables import BUDGETS, SCALES

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nf", list(BUDGETS))
def test_scale_info_matches_kats_and_oracle(nf, gpu, oracle_lib):
    from orb_slam3_ros_amd.extractor import ORBextractor
    ext = ORBextractor(nf, 1.2, 8, 20, 7)
    ref = oracle_lib.OracleExtractor(nf, 1.2, 8, 20, 7).level_info()
    assert ext.GetLevels() == 8
    assert ext.GetScaleFactor() == pytest.approx(1.2, abs=1e-6)
    assert ext.features_per_level == BUDGETS[nf]
    sf = np.array(ext.GetScaleFactors(), np.float32)
    assert np.allclose(sf.astype(np.float64), SCALES, rtol=0, atol=1e-9)
    # float-exact against the restatement (float x double products, 1/x in float)
    for got, key in ((ext.GetScaleFactors(), "scale"), (ext.GetInverseScaleFactors(), "inv_scale"),
                     (ext.GetScaleSigmaSquares(), "sigma2"), (ext.GetInverseScaleSigmaSquares(), "inv_sigma2")):
        g = np.array(got, np.float32)
        assert np.array_equal(g.view(np.uint32), ref[key].view(np.uint32)), key
    ext.close()


@pytest.mark.parametrize("sf,nl", [(1.2, 8), (1.5, 5), (2.0, 3), (1.1, 12)])
def test_scale_info_other_pyramids(sf, nl, gpu, oracle_lib):
    from orb_slam3_ros_amd.extractor import ORBextractor
    ext = ORBextractor(1500, sf, nl, 20, 7)
    ref = oracle_lib.OracleExtractor(1500, sf, nl, 20, 7).level_info()
    assert ext.GetLevels() == nl
    assert ext.features_per_level == ref["per_level"].tolist()
    assert sum(ext.features_per_level) == 1500
    for got, key in ((ext.GetScaleFactors(), "scale"), (ext.GetInverseScaleFactors(), "inv_scale"),
                     (ext.GetScaleSigmaSquares(), "sigma2"), (ext.GetInverseScaleSigmaSquares(), "inv_sigma2")):
        assert np.array_equal(np.array(got, np.float32).view(np.uint32), ref[key].view(np.uint32)), key
    ext.close()
