"""CPU: the field constants compiled into csrc/fp256.hpp are derived from the
moduli of SURVEY.md Appendix A."""
import os
import re

import pasta as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = open(os.path.join(ROOT, "halo2-aggregation_amd", "csrc", "fp256.hpp")).read()


def _struct(name):
    body = re.search(r"struct %s \{(.*?)\n\};" % name, SRC, re.S).group(1)

    def arr(key):
        m = re.search(r"%s\[8\] = \{(.*?)\};" % key, body, re.S)
        return sum(int(x.strip().rstrip("u"), 16) << (32 * i) for i, x in enumerate(m.group(1).split(",")))

    inv = int(re.search(r"INV = (0x[0-9a-f]+)u", body).group(1), 16)
    nbits = int(re.search(r"NBITS = (\d+)", body).group(1))
    return arr("MOD"), inv, arr("ONE"), arr("R2"), nbits


def test_field_constants():
    for name, p in [("PallasFp", P.PALLAS_P), ("VestaFp", P.VESTA_P), ("Bn254Fq", P.BN254_P),
                    ("Bn254Fr", P.BN254_R)]:
        mod, inv, one, r2, nbits = _struct(name)
        assert mod == p, name
        assert inv == (-pow(p, -1, 1 << 32)) % (1 << 32), name
        assert one == P.R_MONT % p, name
        assert r2 == P.R_MONT * P.R_MONT % p, name
        assert nbits == p.bit_length(), name


def _limbs29(src, key):
    m = re.search(r"%s\[9\] = \{(.*?)\};" % key, src, re.S)
    return sum(int(x.strip().rstrip("u"), 16) << (29 * i) for i, x in enumerate(m.group(1).split(",")))


def test_twist_ladder_constants():
    """R522 (canonical -> R = 2^261 Montgomery) and the curves' b in that form:
    the ladder's start point on the twist y^2 = x^3 + A^3 b (accum_kernels.hpp)
    is built from the proof's x bytes with them."""
    fp29 = open(os.path.join(ROOT, "halo2-aggregation_amd", "csrc", "fp29.hpp")).read()
    glv = open(os.path.join(ROOT, "halo2-aggregation_amd", "csrc", "glv.hpp")).read()
    for field, curve, p, b in [("PallasFp", "PallasCurve", P.PALLAS_P, 5), ("VestaFp", "VestaCurve", P.VESTA_P, 5),
                               ("Bn254Fq", "Bn254Curve", P.BN254_P, 3)]:
        body = fp29[fp29.index("struct F29Consts<%s>" % field):]
        assert _limbs29(body, "R522") == pow(2, 522, p), field
        gb = glv[glv.index("struct Glv<%s>" % curve):]
        assert _limbs29(gb, "B29") == b * pow(2, 261, p) % p, curve
