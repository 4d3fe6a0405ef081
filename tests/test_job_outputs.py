"""Output rasters of the local job, CPU side: job.LocalJob with the oracle
engine double (tests/engine_double.py), so the host assembly path (raster.label_rasters /
trendline_rasters) is checked here; tests/test_gpu_job.py checks the GPU assembly
(lt_raster_assemble) against the same literal restatement. Every 'trendline/<date>-<attr>' and
'<rule>_<field>' raster is compared with a literal data2raster over the reducer's per-point
emissions (jobfixture.literal_output_rasters), for an int16 and a uint16 template (numpy 1.x
promotes the uint16 holder to int32)."""
import numpy as np
import pytest

from land_trendr_amd.geotiff import GeoTiff
from land_trendr_amd.job import LocalJob

from engine_double import OracleEngine
from jobfixture import check_job_outputs, make_job


@pytest.mark.parametrize('dtype', [np.int16, np.uint16])
def test_job_output_rasters_match_literal_data2raster(tmp_path, dtype):
    root = str(tmp_path)
    make_job(root, dtype=dtype)
    j = LocalJob(root, 'synth', tile_pixels=40, on_error='skip', engine=OracleEngine())
    files = j.run()
    assert GeoTiff(j.rast_fns[0]).dtype == np.dtype(dtype)
    check_job_outputs(j, files)
