"""Test-side switches of the library: the test hooks (include/skv.h skv_test_option, process-wide,
cleared after every test by conftest.py) and the few environment variables the library still reads
(the host-pipeline thresholds SKV_HOST_PIPE / SKV_HOST_PIPE_MIN / SKV_HOST_PARTS / SKV_SPLIT_PARTS)."""
import os

HOOKS = {"SKV_FUSED", "SKV_SORT", "SKV_FP_TEST", "SKV_FP_GATHER", "SKV_CHUNK_BYTES", "SKV_WAL_FUSED", "SKV_INGEST",
         "SKV_TEST_FAIL_PART", "SKV_PAR_COPY_MIN", "SKV_HI_STEP", "SKV_SPLIT", "SKV_SPLIT_DEBUG", "SKV_SPLIT_SEG",
         "SKV_SPLIT_NC", "SKV_SORT_TWO_PASS", "SKV_SB_NT", "SKV_SB_GMAX", "SKV_FX_TAIL_SLOTS"}


def knob(name, value):
    """set (value) or clear (None) a test hook or a pipeline threshold"""
    if name in HOOKS:
        from skv import api

        api.test_option(name, value)
    elif value is None:
        os.environ.pop(name, None)
    else:
        os.environ[name] = str(value)


def knob_get(name):
    if name in HOOKS:
        from skv import api

        return api.test_option_get(name)
    return os.environ.get(name)
