"""Physical constants used by the synthesis path (values of enterprise.constants, which the
reference vendors as fakepta/constants.py). Only `fyr` enters the hot path (powerlaw PSD)."""
import numpy as np
import scipy.constants as _sc

yr = _sc.Julian_year          # s
day = _sc.day                 # s
fyr = 1.0 / yr                # Hz
c = _sc.speed_of_light
G = _sc.gravitational_constant
AU = _sc.astronomical_unit
pc = _sc.parsec
kpc, Mpc, Gpc = 1e3 * pc, 1e6 * pc, 1e9 * pc
GMsun = 1.327124400e20
Msun = GMsun / G
Tsun = GMsun / c ** 3
pi = np.pi
