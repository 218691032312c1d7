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
