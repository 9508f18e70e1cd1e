"""spectrseqtools_amd -- MI355X-native engine for SpectrSeqTools' per-peak
mass explanation (explain_mass_with_table / is_valid_mass / the packed DP
table), behind the reference's own Python API.

Modules mirror the reference's hot-path modules:
  masses            constants, EXPLANATION_MASSES, build_breakage_dict
  mass_table        DynamicProgrammingTable (table + index resident in HBM)
  mass_explanation  is_valid_mass, explain_mass_with_table, batched explain_masses
  common            Explanation, calculate_explanations
  parallel          spectrum sharding across GPUs + RCCL gather
The compute runs in libsstgpu.so (HIP, gfx950) via the C ABI in include/sst.h.
"""
__version__ = "0.1.0"
