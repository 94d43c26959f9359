/*
 * TEST INFRASTRUCTURE ONLY (tests/conftest.py): names a GPU memory fault.  The HIP runtime turns a
 * GPU page fault into hipErrorIllegalAddress at some later API call without saying where the access
 * went; this registers one more HSA system-event handler that prints, when the fault event arrives,
 * the faulting virtual address, the reason bits, what the HSA runtime knows about that address
 * (hsa_amd_pointer_info: locked host memory, device memory, unknown ...) and the process's CPU
 * mappings around it (/proc/self/maps), so the report of the test that hits it carries the access.
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

static const char* ptype(hsa_amd_pointer_type_t t) {
    switch (t) {
        case HSA_EXT_POINTER_TYPE_UNKNOWN: return "unknown";
        case HSA_EXT_POINTER_TYPE_HSA: return "hsa-allocated";
        case HSA_EXT_POINTER_TYPE_LOCKED: return "locked-host (userptr)";
        case HSA_EXT_POINTER_TYPE_GRAPHICS: return "graphics";
        case HSA_EXT_POINTER_TYPE_IPC: return "ipc";
        default: return "other";
    }
}

static hsa_status_t on_event(const hsa_amd_event_t* e, void* data) {
    (void)data;
    if (!e || e->event_type != HSA_AMD_GPU_MEMORY_FAULT_EVENT) return HSA_STATUS_SUCCESS;
    const uint64_t va = e->memory_fault.virtual_address;
    fprintf(stderr, "FAULT_PROBE: GPU memory fault at va=0x%lx reason_mask=0x%x\n", (unsigned long)va,
            e->memory_fault.fault_reason_mask);
    hsa_amd_pointer_info_t info;
    memset(&info, 0, sizeof(info));
    info.size = sizeof(info);
    if (hsa_amd_pointer_info((void*)(uintptr_t)va, &info, NULL, NULL, NULL) == HSA_STATUS_SUCCESS)
        fprintf(stderr, "FAULT_PROBE: hsa pointer info: type=%s agent_base=%p host_base=%p size=%zu\n",
                ptype(info.type), info.agentBaseAddress, info.hostBaseAddress, (size_t)info.sizeInBytes);
    FILE* f = fopen("/proc/self/maps", "r");
    if (f) {
        char line[512];
        int any = 0;
        while (fgets(line, sizeof line, f)) {
            unsigned long lo = 0, hi = 0;
            if (sscanf(line, "%lx-%lx", &lo, &hi) != 2) continue;
            if (va + (1ul << 22) >= lo && va < hi + (1ul << 22)) {   /* within 4 MiB of the access */
                fprintf(stderr, "FAULT_PROBE: %s %s", va >= lo && va < hi ? "IN  " : "near", line);
                any = 1;
            }
        }
        if (!any) fprintf(stderr, "FAULT_PROBE: no CPU mapping within 4 MiB\n");
        fclose(f);
    }
    fflush(stderr);
    return HSA_STATUS_SUCCESS;
}

/* 0 once the handler is registered (the HSA runtime must be initialised: call after the first HIP call). */
int fault_probe_install(void) { return hsa_amd_register_system_event_handler(on_event, NULL) == HSA_STATUS_SUCCESS ? 0 : -1; }
