"""nremmodfc_amd -- MI355X-native Wilson-Cowan (G, sigma) x seed sweep engine.

Drop-in for the hot path of vandal-uv/NREMmodFC: the Euler-Maruyama loop of
netwWilsonCowanPlastic.py and the sweep drivers whole_sweep_both.py,
whole_sweep_both_maps.py and run_many_seeds.py.  All compute runs in the HIP
library libwcsde.so (csrc/, C ABI in include/wcsde.h).
"""
__version__ = "0.1.0"
