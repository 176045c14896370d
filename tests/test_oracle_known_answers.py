"""Known-answer tests for the oracle rows the reference build cannot pin.

The reference files for these rows (util_mymath.hpp, VD_vehicle_controller.cpp,
VD_motor_if_m2006.cpp, imu_if_wt901c.cpp) need Arduino / CMSIS-DSP / FreeRTOS
headers absent from this image, so they are unbuildable here.  Each expected
value below is derived by hand from the constants and formulas at the cited
reference lines (and from the WIT SDK example, whose scaling matches:
lib/wt901c/examples/wit_c_sdk_normal/wit_c_sdk_normal.ino:54-56).
"""
import numpy as np

from fmskf.synth import wt901_frame

F = np.float32


def test_deg2rad_constant(orc):
    # util_mymath.hpp:14  PI / 180.0f with PI = 3.14159265358979f
    assert orc.deg2rad(1.0) == F(F(3.14159265358979) / F(180.0))
    assert orc.deg2rad(180.0) == F(F(180.0) * F(F(3.14159265358979) / F(180.0)))


def test_normalize_rad(orc):
    two_pi = F(2.0) * F(3.14159265358979)
    assert orc.normalize_rad_0to2pi(0.5) == F(0.5)
    assert orc.normalize_rad_0to2pi(-0.5) == F(F(-0.5) + two_pi)       # mod 0 path, += 2pi
    x = F(7.0)
    assert orc.normalize_rad_0to2pi(7.0) == F(x - F(F(1.0) * F(2.0)) * F(3.14159265358979))
    assert 0.0 <= orc.normalize_rad_0to2pi(-20.0) < float(two_pi)


def test_float_to_int_is_arm_vcvt(orc):
    """The firmware's float -> int casts are Cortex-M7 VCVT (truncate, saturate, NaN -> 0);
    x86's cvttss2si would give 0x80000000 for every out-of-range input."""
    i32max, i32min = 2**31 - 1, -2**31
    for f, want in ((3e9, i32max), (-3e9, i32min), (np.inf, i32max), (-np.inf, i32min),
                    (np.nan, 0), (-2.9, -2), (2147483520.0, 2147483520), (-2147483648.0, i32min)):
        assert orc.f2i32_arm(f) == want, f
    for f, want in ((-1.0, 0), (np.nan, 0), (5e9, 2**32 - 1), (4294967040.0, 4294967040), (7.9, 7)):
        assert orc.f2u32_arm(f) == want, f


def test_normalize_rad_past_2p31_turns(orc):
    # util_mymath.hpp:21 `mod = (int)(d / (2*PI))` saturates on the M7: 1.5e10 rad is 2.39e9
    # turns -> mod = INT32_MAX, d -= (float)mod * 2 * PI (float arithmetic, left to right)
    two_pi = F(2.0) * F(3.14159265358979)
    d = F(1.5e10)
    assert d / two_pi > 2**31
    want = F(d - F(F(F(2**31 - 1) * F(2.0)) * F(3.14159265358979)))
    assert orc.normalize_rad_0to2pi(float(d)) == want
    d = F(-1.5e10)  # mod = INT32_MIN: d -= -2^32 PI, still negative, then += 2 PI
    want = F(d - F(F(F(-2**31) * F(2.0)) * F(3.14159265358979)))
    want = F(want + two_pi) if want < 0 else want
    assert orc.normalize_rad_0to2pi(float(d)) == want
    assert np.isnan(orc.normalize_rad_0to2pi(np.nan))
    assert orc.normalize_rad_0to2pi(np.inf) == np.inf


def test_normalize_deg(orc):
    assert orc.normalize_deg_0to360(-90.0) == F(270.0)
    assert orc.normalize_deg_0to360(725.0) == F(5.0)
    assert orc.normalize_deg_0to360(359.5) == F(359.5)


def test_table512_trig(orc):
    tab = orc.sin_table()
    # CMSIS-DSP sinTable_f32 (arm_common_tables.c) publishes its entries as 8-decimal literals;
    # its first twelve, the peak and the closing -0.00000000f
    cmsis = ["0.00000000", "0.01227154", "0.02454123", "0.03680722", "0.04906767", "0.06132074",
             "0.07356456", "0.08579731", "0.09801714", "0.11022221", "0.12241068", "0.13458071"]
    np.testing.assert_array_equal(tab[:12], np.array([F(float(v)) for v in cmsis]))
    assert tab[128] == F(1.0) and tab[256] == 0.0 and tab[384] == F(-1.0)
    assert tab[512] == 0.0 and np.signbit(tab[512])
    # every entry is sin(2 pi i / 512) rounded to 8 decimals, then to float: 62 of them differ
    # by 1-2 ulp from (float)sin(2 pi i / 512)
    lit = np.array([F(float(f"{np.sin(2 * np.pi * i / 512):.8f}")) for i in range(513)])
    np.testing.assert_array_equal(tab, lit)
    assert int((tab != np.sin(2 * np.pi * np.arange(513) / 512).astype(np.float32)).sum()) == 62
    # exact at table nodes: x = 2*pi*k/512 -> in = k/512 up to rounding
    x = np.linspace(-10, 10, 20001).astype(np.float32)
    s, c = orc.eval_trig(x, orc.TRIG_TABLE512)
    assert np.abs(s - np.sin(x.astype(np.float64))).max() < 2.5e-5   # CMSIS-style lerp error
    assert np.abs(c - np.cos(x.astype(np.float64))).max() < 2.5e-5
    sl, cl = orc.eval_trig(x, orc.TRIG_LIBM)
    assert np.abs(sl - np.sin(x.astype(np.float64))).max() < 1e-6


def test_mecanum_fk_known_answers(orc):
    # VD_vehicle_controller.cpp:126-130, R = 37.5 mm
    v = orc.mdir_to_vdir([1, 1, 1, 1])          # all wheels forward 1 rad -> x = R
    assert v[0] == F(37.5) and v[1] == 0 and v[2] == 0
    v = orc.mdir_to_vdir([-1, 1, -1, 1])        # strafe left -> y = R
    assert v[0] == 0 and v[1] == F(37.5)
    v = orc.mdir_to_vdir([-1, -1, 1, 1])        # rotate CCW
    expect = F(F(F(F(4.0) * F(0.25)) / F(1.41421356)) / F(13.08148)) * F(37.5)
    assert v[2] == expect


def test_wt901_yaw_known_answer(orc):
    # Yaw register 0x2000 -> 0x2000/32768*180 = 45 deg (imu_if_wt901c.cpp:99)
    w = orc.Wt901(0x51)
    q = wt901_frame(0x59, [0x4000, 0, 0, 0x4000])
    w.update(wt901_frame(0x53, [0, 0, 0x2000, 0]) + q)
    assert not w.is_error
    d = w.data
    assert d[11] == F(45.0)
    assert d[9] == F(F(0.0) - F(180.0)) + F(360.0) - F(360.0) or d[9] == F(-180.0)  # roll 0 -> normalize -> -180
    # q_init is zero before the init latch -> relative quaternion is zero
    assert np.all(d[12:16] == 0)


def test_wt901_quaternion_product(orc):
    # init(): latch q_init = q (imu_if_wt901c.cpp:70-76); then the relative quaternion of the
    # same attitude is the identity (0, 0, 0, 1) in x,y,z,w order (:123-126)
    w = orc.Wt901(0x51)
    q = [0x2000, 0x1000, 0x0800, 0x6000]
    w.update(wt901_frame(0x59, q), latch_qinit=True)
    w.update(wt901_frame(0x59, q))
    d = w.data
    qq = np.array(q, np.float32) / F(32768.0)
    assert abs(d[15] - float(np.dot(qq, qq))) < 1e-6
    assert np.abs(d[12:15]).max() < 1e-7


def test_wt901_error_without_quaternion(orc):
    # isComComp is true only if a quaternion frame arrived (imu_if_wt901c.cpp:138-142)
    w = orc.Wt901(0x51)
    w.update(wt901_frame(0x53, [1, 2, 3, 4]))
    assert w.is_error
    w.update(wt901_frame(0x59, [1, 2, 3, 4]))
    assert not w.is_error
    assert w.data[11] == F(F(3.0) / F(32768.0)) * F(180.0)  # stale angle frame applied now


def test_m2006_unwrap(orc):
    # VD_motor_if_m2006.cpp:66-69: 13-bit wrap into the int64 sum
    m = orc.M2006(1)
    seq = [8000, 8150, 10, 200, 8100, 4000]
    stamps = [100, 1100, 2100, 3100, 4100, 5100]
    sums = []
    for a, st in zip(seq, stamps):
        m.rx(bytes([a >> 8, a & 0xFF, 0, 100, 0, 50, 0, 0]), st)
        sums.append(m.s.angle_sum)
    # first frame: delta from the zero-initialised status (8000 > 4096 -> -192)
    # 8100 -> 4000 is -4100 < -4096 -> wrapped to +4092
    assert sums == [-192, -42, -42 + 52, -42 + 52 + 190, -42 + 52 + 190 - 292,
                    -42 + 52 + 190 - 292 + 4092]
    assert m.s.rpm == 100 and m.s.curr == 50


def test_m2006_reversed_motor(orc):
    # dir = -1: angle = 8192 - raw, rpm/current negated (VD_motor_if_m2006.cpp:39-46)
    m = orc.M2006(-1)
    m.rx(bytes([0, 10, 0x01, 0x00, 0xFF, 0x38, 0, 0]), 500)
    assert m.s.angle == 8182 and m.s.rpm == -256 and m.s.curr == 200


def test_m2006_speed_arm_semantics(orc):
    # equal stamps -> usec_dlt == 0 -> Cortex-M7 SDIV returns 0 (x86 would trap)
    m = orc.M2006(1)
    m.rx(bytes([0, 100, 0, 0, 0, 0, 0, 0]), 1000)
    m.rx(bytes([0, 200, 0, 0, 0, 0, 0, 0]), 1000)
    assert np.isfinite(m.s.speed_radps)


def test_rs_tick_straight_line(orc):
    # all four wheels advance d counts -> Mrad = d*OUT_RAD/36 (double), x += R*Mrad*0.001
    n = 1
    pos = np.zeros((3, n), np.float32)
    vel = np.zeros((3, n), np.float32)
    prev = np.zeros((4, n), np.int64)
    sums = np.full((4, n), 100, np.int64)
    rpm = np.zeros((n, 4), np.int16)
    orc.rs_tick(pos, vel, prev, np.zeros(n, np.float32), sums, rpm)
    out_rad = F(F(F(2.0) * F(3.1415926)) / F(8191.0))
    mrad = F(float(100.0) * float(out_rad) * float(F(1.0) / F(36.0)))
    lx = F(F(F(F(F(F(mrad) + mrad) + mrad) + mrad) * F(0.25)) * F(37.5))
    assert pos[0, 0] == F(F(0.0) + F(F(lx * F(1.0) - F(0.0) * F(0.0)) * F(0.001)))
    assert pos[1, 0] == 0.0
    assert np.all(prev == sums)


def test_rs_correct_overwrites_theta(orc):
    pos = np.zeros((3, 2), np.float32)
    vel = np.zeros((3, 2), np.float32)
    prev = np.zeros((4, 2), np.int64)
    orc.rs_tick(pos, vel, prev, np.array([90.0, -45.0], np.float32), prev.copy(),
                np.zeros((2, 4), np.int16), do_predict=False)
    d2r = F(F(3.14159265358979) / F(180.0))
    assert pos[2, 0] == F(F(90.0) * d2r) and pos[2, 1] == F(F(-45.0) * d2r)
