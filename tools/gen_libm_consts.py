"""Constants of ndt_libm.h (exp_dr, sincosf_dr), computed with Python's decimal module at 80 digits: the 2^(i/64)
double-double table, 64/ln2, ln2/64 split for a Cody-Waite reduction (hi with 39 significant bits), pi/2 split 33/33/rest,
and the Taylor coefficients.  Run: python tools/gen_libm_consts.py"""
from decimal import Decimal, getcontext
import struct
getcontext().prec = 80
ln2 = Decimal(2).ln()
def bits(f): return struct.unpack('<Q', struct.pack('<d', f))[0]
rows=[]
for i in range(64):
    v = (ln2 * i / 64).exp()
    hi = float(v)
    lo = float(v - Decimal(hi))
    rows.append((hi, lo))
print("table")
for i in range(0,64,2):
    print("    %s, %s, %s, %s," % tuple(hex(bits(x))+"ull" for x in (rows[i][0], rows[i][1], rows[i+1][0], rows[i+1][1])))
inv = float(Decimal(64)/ln2)
print("InvLn2N", inv.hex())
c = ln2/64
# hi: 39 significant bits
import math
h = float(c)
m, e = math.frexp(h)
hi39 = math.ldexp(math.floor(m * 2**39), e-39)
lo = float(c - Decimal(hi39))
print("Ln2hiN", hi39.hex(), "Ln2loN", lo.hex())
# pi/2 split 33/33/rest
pi = Decimal('3.14159265358979323846264338327950288419716939937510582097494459230781640628620899862803482534211706798214808651')
p2 = pi/2
def trunc_bits(d, nb):
    f = float(d); m, e = math.frexp(f)
    t = math.ldexp(math.floor(m*2**nb), e-nb)
    # make sure truncation is exact w.r.t decimal (floor of real value)
    return t
P1 = trunc_bits(p2, 33); r1 = p2 - Decimal(P1)
P2 = trunc_bits(r1, 33); r2 = r1 - Decimal(P2)
P3 = float(r2)
print("P1", P1.hex(), "P2", P2.hex(), "P3", P3.hex(), "2/pi", float(2/pi).hex())
for k in range(2,7): print("1/%d!"%k, float(Decimal(1)/math.factorial(k)).hex())
for k in range(3,20,2): print("sin 1/%d!"%k, float(Decimal(1)/math.factorial(k)).hex())
for k in range(2,21,2): print("cos 1/%d!"%k, float(Decimal(1)/math.factorial(k)).hex())
