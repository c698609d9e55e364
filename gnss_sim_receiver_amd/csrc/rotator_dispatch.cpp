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
// with the largest arch requirement the CPU meets: u_avx/a_avx on an AVX host).  The unaligned
// entry is read (the tracking input is a GNU Radio buffer at an arbitrary offset); generic_reload
// maps to generic.
extern "C" int gnsship_rotator_dispatch(int* variant)
{
    if (!variant) return GNSSHIP_E_INVAL;
    if (std::getenv("VOLK_GENERIC")) {
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
        int found = -1;
        while (std::fgets(line, sizeof(line), f)) {
            if (std::sscanf(line, "%511s %511s %511s", name, impl_a, impl_u) == 3 &&
                std::strcmp(name, "volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn") == 0)
                found = std::strstr(impl_u, "avx") ? GNSSHIP_ROTATOR_AVX : GNSSHIP_ROTATOR_GENERIC;
        }
        std::fclose(f);
        if (found >= 0) {
            *variant = found;
            return GNSSHIP_OK;
        }
        break;
    }
    __builtin_cpu_init();
    *variant = __builtin_cpu_supports("avx") ? GNSSHIP_ROTATOR_AVX : GNSSHIP_ROTATOR_GENERIC;
    return GNSSHIP_OK;
}
