"""Import-only stand-in for `ms_deisotope` (absent; RAW preprocessing is out of
scope).  TEST INFRASTRUCTURE ONLY: common.py imports it and names
ms_deisotope.data_source.thermo_raw_net.ThermoRawLoader in an annotation."""
import types


class ThermoRawLoader:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("ms_deisotope stand-in: RAW reading is not available in this container")


data_source = types.SimpleNamespace(thermo_raw_net=types.SimpleNamespace(ThermoRawLoader=ThermoRawLoader))
