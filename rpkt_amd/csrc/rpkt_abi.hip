// rpkt_abi.hip — host-only entry points of the C ABI (version, build info, status names,
// device info) and the per-thread last-HIP-error slot.
#include "rpkt_common.h"

namespace rpkt_detail {
thread_local int g_last_hip_error = 0;
}  // namespace rpkt_detail

using rpkt_detail::g_last_hip_error;

extern "C" {

uint32_t rpkt_gpu_abi_version(void) { return RPKT_ABI_VERSION; }

#ifndef RPKT_SRC_HASH
#define RPKT_SRC_HASH "dev"
#endif
#ifndef RPKT_UNIT_HASHES
#define RPKT_UNIT_HASHES "dev"
#endif
const char* rpkt_gpu_build_info(void) {
    return "rpkt_gpu src=" RPKT_SRC_HASH " gfx950; rec=80B; tile=64 frames/wave; win=128B; "
           RPKT_UNIT_HASHES;
}

const char* rpkt_gpu_status_name(int s) {
    static const char* names[] = {"OK", "ETH_SHORT", "VLAN_SHORT", "NOT_IPV4", "IP_SHORT",
                                  "IP_BAD_IHL", "IP_IHL_GT_LEN", "IP_TOT_LT_IHL",
                                  "IP_TOT_GT_LEN", "L4_OTHER", "UDP_SHORT", "UDP_BAD_LEN",
                                  "TCP_SHORT", "TCP_BAD_DOFF", "IP6_SHORT", "IP6_BAD_LEN",
                                  "IP6_EXT_SHORT", "IP6_EXT_BAD_LEN", "IP6_FRAGMENT",
                                  "ICMP_EMPTY", "NO_INNER"};
    return (s >= 0 && s < (int)(sizeof(names) / sizeof(names[0]))) ? names[s] : "?";
}

int rpkt_gpu_last_hip_error(void) { return g_last_hip_error; }

int rpkt_gpu_device_info(char* buf, size_t len) {
    int count = 0, dev = -1;
    hipError_t e1 = hipGetDeviceCount(&count);
    hipError_t e2 = hipGetDevice(&dev);
    hipDeviceProp_t p;
    memset(&p, 0, sizeof(p));
    hipError_t e3 = dev >= 0 ? hipGetDeviceProperties(&p, dev) : hipErrorInvalidDevice;
    int rv = 0;
    if (hipRuntimeGetVersion(&rv) != hipSuccess) rv = -1;
    if (buf && len)
        snprintf(buf, len, "hip_runtime=%d devices=%d(err %d) current=%d(err %d) name=%s arch=%s "
                 "cus=%d (err %d)", rv, count, (int)e1, dev, (int)e2, p.name, p.gcnArchName,
                 p.multiProcessorCount, (int)e3);
    return (e1 == hipSuccess && count > 0) ? RPKT_OK : RPKT_E_HIP;
}

}  // extern "C"
