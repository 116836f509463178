"""Optical materials with wavelength-dependent refractive index -- drop-in for ``raytrace.materials``.

Same classes, constructor signatures, attributes (``b1..b3``, ``c1..c3``, ``vd``, ``wd/wf/wc``) and
``n(wavelength)`` semantics as the reference (QI2lab/ray_trace_pb @ 2024_10_08,
src/raytrace/materials.py = MAT).  ``n`` here is the host-side evaluation used by the paraxial API and
by user code; inside ``System.ray_trace`` the GPU kernel evaluates n(lambda) per ray itself from the
descriptor each material lowers to (:meth:`Material._rtpb_lower`):

* Sellmeier ``Material`` (incl. ``Vacuum`` and the glass catalogue)  -> RTPB_SELLMEIER  (MAT:39-51)
* ``Constant``                                                          -> RTPB_CONSTANT   (MAT:59-79)
* ``Ebaf11`` (6-term polynomial in lambda^2, lambda^-2k, MAT:128-144) and any user subclass that
  overrides ``n`` (the reference's documented plugin point, MAT:39-44) -> RTPB_TABLE: ``n`` is
  evaluated on the host, by the material's own NumPy code, at the distinct wavelengths of the ray
  bundle and the kernel looks each ray's value up (binary search), so arbitrary dispersion laws trace
  on the GPU with the reference's exact values.  (Ebaf11 is not sent as RTPB_POLY6: NumPy's SIMD
  ``power`` and the device ``pow`` disagree in the last bit on ~5 % of wavelengths.)
"""
import numpy as np

from . import _engine as _E

# (b1, b2, b3), (c1, c2, c3) Sellmeier coefficients, wavelength in um (Schott / refractiveindex.info)
_SELLMEIER = {
    "FusedSilica": ((0.6961663, 0.4079426, 0.8974794), (0.0684043 ** 2, 0.1162414 ** 2, 9.896161 ** 2)),
    "Bk7": ((1.03961212, 0.231792344, 1.01046945), (0.00600069867, 0.0200179144, 103.560653)),
    "Nbak4": ((1.28834642, 0.132817724, 0.945395373), (0.00779980626, 0.0315631177, 105.965875)),
    "Nbaf10": ((1.5851495, 0.143559385, 1.08521269), (0.00926681282, 0.0424489805, 105.613573)),
    "Nlak22": ((1.14229781, 0.535138441, 1.040883850), (0.00585778594, 0.0198546147, 100.8340170)),
    "Nsk11": ((1.17963631, 0.229817295, 0.935789652), (0.00680282081, 0.0219737205, 101.513232)),
    "Sf10": ((1.62153902, 0.256287842, 1.64447552), (0.0122241457, 0.0595736775, 147.468793)),
    "Nsf11": ((1.737596950, 0.313747346, 1.898781010), (0.013188707, 0.0623068142, 155.23629000)),
    "Nsf6": ((1.77931763, 0.338149866, 2.087344740), (0.01337141820, 0.0617533621, 174.0175900)),
    "Sf6": ((1.72448482, 0.390104889, 1.045728580), (0.01348719470, 0.0569318095, 118.5571850)),
    "Nsf6ht": ((1.77931763, 0.338149866, 2.087344740), (0.01337141820, 0.0617533621, 174.0175900)),
    "Sf2": ((1.40301821, 0.231767504, 0.939056586), (0.0105795466, 0.0493226978, 112.405955)),
    "Nsf19": ((1.52005444, 0.17573947, 1.43623424), (0.01096144, 0.0593248486, 126.795151)),
}

# Ebaf11 (HIKARI E-BAF11): n^2 = p0 + p1 w^2 + p2 w^-2 + p3 w^-4 + p4 w^-6 + p5 w^-8
_EBAF11 = (2.71954649, -0.0100472501, 0.0200301385, 0.00046586302, -7.51633336e-6, 1.77544989e-6)

# lowering kinds (include/rtpb.h)
RTPB_CONSTANT, RTPB_SELLMEIER, RTPB_POLY6, RTPB_TABLE = 0, 1, 2, 3


class Material:
    """Sellmeier material: n^2 = 1 + sum_k b_k w^2 / (w^2 - c_k)  (MAT:6-51).

    Abbe number ``vd = (n_d - 1) / (n_F - n_C)``; ``vd > 50`` = crown glass, otherwise flint.
    Subclass and override :meth:`n` to define another dispersion law."""

    wd = 0.5876   # helium d-line
    wf = 0.4861   # hydrogen F-line
    wc = 0.6563   # hydrogen C-line
    vd = None

    # every assignment / deletion of an attribute is counted: the drop-in call's lowering memo is valid only while
    # the count is unchanged (_engine.memo_lookup)
    def __setattr__(self, name, value):
        object.__setattr__(self, name, value)
        _E.MUTATIONS[0] += 1

    def __delattr__(self, name):
        object.__delattr__(self, name)
        _E.MUTATIONS[0] += 1

    def __init__(self, b_coeffs, c_coeffs):
        self.b1, self.b2, self.b3 = np.array(b_coeffs).squeeze()
        self.c1, self.c2, self.c3 = np.array(c_coeffs).squeeze()
        with np.errstate(invalid="ignore", divide="ignore"):
            self.vd = (self.n(self.wd) - 1) / (self.n(self.wf) - self.n(self.wc))

    def n(self, wavelength):
        """Refractive index at ``wavelength`` (um); scalar or array."""
        w2 = wavelength ** 2
        val = self.b1 * w2 / (w2 - self.c1) + self.b2 * w2 / (w2 - self.c2) + self.b3 * w2 / (w2 - self.c3)
        return np.sqrt(val + 1)

    # ---- lowering to the C ABI descriptor (kind, 6 coefficients) or None for a per-wavelength table
    def _rtpb_lower(self):
        if type(self).n is Material.n:
            return RTPB_SELLMEIER, (self.b1, self.b2, self.b3, self.c1, self.c2, self.c3)
        return None

    def __repr__(self):
        return f"{type(self).__name__}()"


class Vacuum(Material):
    """n = 1 (Sellmeier with zero coefficients, MAT:54-56)."""

    def __init__(self):
        super().__init__([0., 0., 0.], [0., 0., 0.])


class Constant(Material):
    """Wavelength-independent index (MAT:59-79)."""

    def __init__(self, n):
        self._n = float(n)
        self.b1 = self.b2 = self.b3 = None
        self.c1 = self.c2 = self.c3 = None

    def n(self, wavelength: float):
        if isinstance(wavelength, float):
            return self._n
        wavelength = np.atleast_1d(np.array(wavelength))
        return np.ones(wavelength.shape) * self._n

    def _rtpb_lower(self):
        if type(self).n is Constant.n:
            return RTPB_CONSTANT, (self._n, 0., 0., 0., 0., 0.)
        return None

    def __repr__(self):
        return f"Constant({self._n!r})"


class Ebaf11(Material):
    """HIKARI E-BAF11, 6-term polynomial dispersion (MAT:128-144)."""

    def __init__(self):
        self.params = list(_EBAF11)

    def n(self, wavelength):
        p = self.params
        n_sqr = (p[0] + p[1] * wavelength ** 2 + p[2] * wavelength ** -2 + p[3] * wavelength ** -4 +
                 p[4] * wavelength ** -6 + p[5] * wavelength ** -8)
        return np.sqrt(n_sqr)

    def _rtpb_lower(self):
        # Lowered as a host-evaluated (wavelength, n) table, not RTPB_POLY6: NumPy evaluates
        # wavelength**-2k with its SIMD power, which differs from libm/device pow() in the last bit
        # on ~5 % of wavelengths (AVX-512 hosts), and bit-exactness needs the reference's own n().
        return None

    def _rtpb_table_key(self):
        # everything n() reads (the lowering memo and the previous-bundle key cache are keyed by it)
        return tuple(float(p) for p in self.params)


def _glass(name, doc):
    b, c = _SELLMEIER[name]

    def __init__(self):
        Material.__init__(self, b, c)
    return type(name, (Material,), {"__init__": __init__, "__doc__": doc, "__module__": __name__})


FusedSilica = _glass("FusedSilica", "Fused silica.")
Bk7 = _glass("Bk7", "BK7 crown glass.")
Nbak4 = _glass("Nbak4", "N-BAK4 crown glass.")
Nbaf10 = _glass("Nbaf10", "N-BAF10 crown glass.")
Nlak22 = _glass("Nlak22", "N-LAK22 crown glass.")
Nsk11 = _glass("Nsk11", "N-SK11 crown glass.")
Sf10 = _glass("Sf10", "SF10 flint glass.")
Nsf11 = _glass("Nsf11", "N-SF11 flint glass.")
Nsf6 = _glass("Nsf6", "N-SF6 flint glass.")
Sf6 = _glass("Sf6", "SF6 flint glass.")
Nsf6ht = _glass("Nsf6ht", "N-SF6HT flint glass.")
Sf2 = _glass("Sf2", "SF2 flint glass.")
Nsf19 = _glass("Nsf19", "N-SF19 flint glass.")

__all__ = ["Material", "Vacuum", "Constant", "Ebaf11"] + list(_SELLMEIER)
