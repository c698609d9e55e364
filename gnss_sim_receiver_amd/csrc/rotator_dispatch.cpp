// rotator_dispatch.cpp — host C++ (no device code): which volk_gnsssdr rotator variant the
// reference would run on this machine (include/gnsship.h gnsship_rotator_dispatch).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "gnsship.h"

// volk_gnsssdr's dispatch of volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn on this host
// (volk_gnsssdr_rank_archs.c: VOLK_GENERIC → "generic"; else a volk_gnsssdr_prefs.c preferences
// entry — $VOLK_CONFIGPATH/volk_gnsssdr/volk_gnsssdr_config, then $HOME/.volk_gnsssdr/volk_gnsssdr_config,
// then /etc/volk_gnsssdr/volk_gnsssdr_config, lines "name impl_a impl_u" — else the implementation
// with the largest arch requirement the CPU meets: u_avx/a_avx on an AVX host).  The reference takes
// impl_a for aligned buffers and impl_u otherwise (volk_gnsssdr_rank_archs.c:71); both must name a
// variant the engine reproduces and the same one (generic, or a_avx / u_avx).  Any other entry —
// generic_reload (renormalises after every 256 samples instead of before) or an SSE / AVX2 variant —
// is reported as unsupported rather than mapped to the nearest one.
namespace {
thread_local std::string g_detail;

int classify(const char* impl)
{
    if (std::strcmp(impl, "generic") == 0) return GNSSHIP_ROTATOR_GENERIC;
    if (std::strcmp(impl, "u_avx") == 0 || std::strcmp(impl, "a_avx") == 0) return GNSSHIP_ROTATOR_AVX;
    return -1;
}
}  // namespace

extern "C" int gnsship_rotator_dispatch(int* variant)
{
    if (!variant) return GNSSHIP_E_INVAL;
    if (std::getenv("VOLK_GENERIC")) {
        g_detail = "VOLK_GENERIC is set: generic";
        *variant = GNSSHIP_ROTATOR_GENERIC;
        return GNSSHIP_OK;
    }
    std::string paths[3];
    if (const char* c = std::getenv("VOLK_CONFIGPATH")) paths[0] = std::string(c) + "/volk_gnsssdr/volk_gnsssdr_config";
    if (const char* h = std::getenv("HOME")) paths[1] = std::string(h) + "/.volk_gnsssdr/volk_gnsssdr_config";
    paths[2] = "/etc/volk_gnsssdr/volk_gnsssdr_config";
    for (const auto& path : paths) {
        if (path.empty()) continue;
        FILE* f = std::fopen(path.c_str(), "r");
        if (!f) continue;  // the reference takes the first file that exists
        char line[512], name[512], impl_a[512], impl_u[512];
        std::string entry_a, entry_u;
        while (std::fgets(line, sizeof(line), f)) {
            if (std::sscanf(line, "%511s %511s %511s", name, impl_a, impl_u) == 3 &&
                std::strcmp(name, "volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn") == 0) {
                entry_a = impl_a;
                entry_u = impl_u;
            }
        }
        std::fclose(f);
        if (!entry_u.empty()) {
            const int va = classify(entry_a.c_str()), vu = classify(entry_u.c_str());
            g_detail = path + ": " + entry_a + " " + entry_u;
            if (va < 0 || vu < 0 || va != vu) {
                g_detail += " (not a variant the engine reproduces: generic, a_avx / u_avx)";
                return GNSSHIP_E_INVAL;
            }
            *variant = vu;
            return GNSSHIP_OK;
        }
        break;
    }
    __builtin_cpu_init();
    const bool avx = __builtin_cpu_supports("avx");
    g_detail = avx ? "no preferences entry; the CPU has AVX: u_avx/a_avx" : "no preferences entry; no AVX: generic";
    *variant = avx ? GNSSHIP_ROTATOR_AVX : GNSSHIP_ROTATOR_GENERIC;
    return GNSSHIP_OK;
}

extern "C" int gnsship_rotator_dispatch_detail(char* buf, int cap)
{
    if (!buf || cap < 1) return GNSSHIP_E_INVAL;
    std::snprintf(buf, static_cast<size_t>(cap), "%s", g_detail.c_str());
    return GNSSHIP_OK;
}
