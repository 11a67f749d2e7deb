// java_compat.h — the JDK 17 / JOML 1.10.7 / java.awt behaviours the reference's
// scene code depends on, restated in C++ (host-only; built with
// -ffp-contract=off so float expressions round like Java's strict IEEE floats).
#pragma once

#include <cmath>
#include <cstdint>

namespace rtb {

// Java's (int) of a float or double (JLS 5.1.3): NaN -> 0, out of range -> Integer.MIN / MAX_VALUE,
// else truncation -- the C++ cast for every in-range value, without its undefined behaviour outside.
inline int32_t java_f2i(double x) {
    if (x != x) return 0;
    if (x >= 2147483647.0) return INT32_MAX;
    if (x <= -2147483648.0) return INT32_MIN;
    return (int32_t)x;
}

// java.util.Random (48-bit LCG), JDK 17 semantics.
struct JavaRandom {
    static constexpr uint64_t kMul = 0x5DEECE66DULL;
    static constexpr uint64_t kMask = (1ULL << 48) - 1;
    uint64_t seed;
    explicit JavaRandom(int64_t s) { set_seed(s); }
    void set_seed(int64_t s) { seed = ((uint64_t)s ^ kMul) & kMask; }
    int32_t next(int bits) {
        seed = (seed * kMul + 0xBULL) & kMask;
        return (int32_t)(uint32_t)(seed >> (48 - bits));
    }
    int32_t next_int() { return next(32); }
    // Random.nextInt(int bound)
    int32_t next_int(int32_t bound) {
        int32_t r = next(31);
        int32_t m = bound - 1;
        if ((bound & m) == 0) return (int32_t)(((int64_t)bound * (int64_t)r) >> 31);
        for (int32_t u = r; (int32_t)((uint32_t)u - (uint32_t)(r = u % bound) + (uint32_t)m) < 0; u = next(31)) {
        }
        return r;
    }
    float next_float() { return (float)next(24) / (float)(1 << 24); }
    double next_double() {
        int64_t hi = (int64_t)next(26);
        int64_t lo = (int64_t)next(27);
        return (double)((hi << 27) + lo) * 0x1.0p-53;
    }
    // RandomGenerator.nextFloat(origin, bound) -> RandomSupport.boundedNextFloat
    float next_float(float origin, float bound) {
        float r = next_float();
        if (origin < bound) {
            r = r * (bound - origin) + origin;
            if (r >= bound) r = std::nextafter(bound, -INFINITY);
        }
        return r;
    }
};

// org.joml.Vector3f subset (non-FMA JOML build: Math.fma(a,b,c) == a*b+c).
struct Vec3f {
    float x = 0, y = 0, z = 0;
    Vec3f() = default;
    Vec3f(float a, float b, float c) : x(a), y(b), z(c) {}
    explicit Vec3f(float s) : x(s), y(s), z(s) {}
    Vec3f add(const Vec3f& v) const { return {x + v.x, y + v.y, z + v.z}; }
    Vec3f add(float a, float b, float c) const { return {x + a, y + b, z + c}; }
    Vec3f sub(const Vec3f& v) const { return {x - v.x, y - v.y, z - v.z}; }
    Vec3f sub(float a, float b, float c) const { return {x - a, y - b, z - c}; }
    Vec3f mul(float s) const { return {x * s, y * s, z * s}; }
    Vec3f div(float s) const { float inv = 1.0f / s; return {x * inv, y * inv, z * inv}; }
    Vec3f negate() const { return {-x, -y, -z}; }
    // Vector3f.cross: rx = fma(y, v.z, -z*v.y) ...
    Vec3f cross(const Vec3f& v) const {
        return {y * v.z + (-z * v.y), z * v.x + (-x * v.z), x * v.y + (-y * v.x)};
    }
    float dot(const Vec3f& v) const { return x * v.x + (y * v.y + z * v.z); }
    float length_squared() const { return x * x + (y * y + z * z); }
    float length() const { return (float)std::sqrt((double)length_squared()); }
    // Vector3f.normalize: scalar = invsqrt(lenSq) = 1/(float)sqrt(lenSq)
    Vec3f normalize() const {
        float s = 1.0f / (float)std::sqrt((double)length_squared());
        return {x * s, y * s, z * s};
    }
};

// org.joml.Matrix3f subset: column-major mCR (column C, row R).
struct Mat3f {
    float m00 = 1, m01 = 0, m02 = 0, m10 = 0, m11 = 1, m12 = 0, m20 = 0, m21 = 0, m22 = 1;
    static float jsin(float a) { return (float)std::sin((double)a); }
    // org.joml.Math.cosFromSin (non-FASTMATH)
    static float cos_from_sin(float sin, float angle) {
        const float PIHalf_f = (float)(M_PI * 0.5);
        const float PI2_f = (float)(M_PI * 2.0);
        const float PI_f = (float)M_PI;
        float cos = (float)std::sqrt((double)(1.0f - sin * sin));
        float a = angle + PIHalf_f;
        float b = a - (float)java_f2i(a / PI2_f) * PI2_f;
        if (b < 0.0) b = PI2_f + b;
        if (b >= PI_f) return -cos;
        return cos;
    }
    Mat3f rotate_x(float ang) const {
        float s = jsin(ang), c = cos_from_sin(s, ang);
        float rm11 = c, rm21 = -s, rm12 = s, rm22 = c;
        Mat3f d = *this;
        float nm10 = m10 * rm11 + m20 * rm12, nm11 = m11 * rm11 + m21 * rm12, nm12 = m12 * rm11 + m22 * rm12;
        d.m20 = m10 * rm21 + m20 * rm22; d.m21 = m11 * rm21 + m21 * rm22; d.m22 = m12 * rm21 + m22 * rm22;
        d.m10 = nm10; d.m11 = nm11; d.m12 = nm12;
        return d;
    }
    Mat3f rotate_y(float ang) const {
        float s = jsin(ang), c = cos_from_sin(s, ang);
        float rm00 = c, rm20 = s, rm02 = -s, rm22 = c;
        Mat3f d = *this;
        float nm00 = m00 * rm00 + m20 * rm02, nm01 = m01 * rm00 + m21 * rm02, nm02 = m02 * rm00 + m22 * rm02;
        d.m20 = m00 * rm20 + m20 * rm22; d.m21 = m01 * rm20 + m21 * rm22; d.m22 = m02 * rm20 + m22 * rm22;
        d.m00 = nm00; d.m01 = nm01; d.m02 = nm02;
        return d;
    }
    Mat3f rotate_z(float ang) const {
        float s = jsin(ang), c = cos_from_sin(s, ang);
        float rm00 = c, rm10 = -s, rm01 = s, rm11 = c;
        Mat3f d = *this;
        float nm00 = m00 * rm00 + m10 * rm01, nm01 = m01 * rm00 + m11 * rm01, nm02 = m02 * rm00 + m12 * rm01;
        d.m10 = m00 * rm10 + m10 * rm11; d.m11 = m01 * rm10 + m11 * rm11; d.m12 = m02 * rm10 + m12 * rm11;
        d.m00 = nm00; d.m01 = nm01; d.m02 = nm02;
        return d;
    }
    // Vector3f.mul(Matrix3fc) = M * v
    Vec3f transform(const Vec3f& v) const {
        return {m00 * v.x + (m10 * v.y + m20 * v.z), m01 * v.x + (m11 * v.y + m21 * v.z),
                m02 * v.x + (m12 * v.y + m22 * v.z)};
    }
};

// java.awt.Color(float r, float g, float b): (int)(r*255+0.5) per channel.
struct AwtColor {
    int r = 0, g = 0, b = 0;
    static int chan(float f) { return java_f2i((double)(f * 255.0f) + 0.5); }
    static bool valid(float f) { return f >= 0.0f && f <= 1.0f; }
};

// Math.toRadians (JDK 9+): angdeg * (PI/180)
inline double to_radians(double deg) { return deg * 0.017453292519943295; }

}  // namespace rtb
