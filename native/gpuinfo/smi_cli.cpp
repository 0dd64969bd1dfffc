// gpushare-smi — command-line view of libgpushare_gpuinfo (the MI355X replacement for the
// NVML queries the reference makes at startup, nvidia.go:50-86).
//   gpushare-smi [--backend SPEC] [--json] [--events SECONDS]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "gpuinfo.h"

static const char* link_name(int t) {
  switch (t) {
    case GS_LINK_XGMI: return "XGMI";
    case GS_LINK_PCIE: return "PCIE";
    case GS_LINK_SELF: return "SELF";
    default: return "NONE";
  }
}

int main(int argc, char** argv) {
  std::string spec = "auto";
  bool json = false;
  int events_s = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--backend") && i + 1 < argc) spec = argv[++i];
    else if (!strcmp(argv[i], "--json")) json = true;
    else if (!strcmp(argv[i], "--events") && i + 1 < argc) events_s = atoi(argv[++i]);
    else {
      fprintf(stderr, "usage: %s [--backend auto|rocm_smi|sysfs[:root]|fake:SPEC] [--json] [--events S]\n", argv[0]);
      return 2;
    }
  }
  gs_handle* h = nullptr;
  if (gs_open(spec.c_str(), &h) != 0) {
    fprintf(stderr, "gpushare-smi: %s\n", gs_last_error());
    return 1;
  }
  if (json) {
    int n = gs_to_json(h, nullptr, 0);
    std::vector<char> buf((size_t)n + 1);
    gs_to_json(h, buf.data(), buf.size());
    printf("%s\n", buf.data());
  } else {
    int n = gs_device_count(h);
    printf("backend: %s  devices: %d  inaccessible: %d\n", gs_backend_name(h), n, gs_inaccessible_count(h));
    printf("%-3s %-22s %-13s %-7s %-10s %-5s %-5s %-4s %s\n", "IDX", "UUID", "BDF", "GFX", "VRAM(GiB)", "NUMA",
           "REND", "PART", "NAME");
    for (int i = 0; i < n; ++i) {
      gs_device_t d;
      gs_get_device(h, i, &d);
      printf("%-3d %-22s %-13s %-7s %-10.2f %-5d %-5d %d/%d  %s\n", d.index, d.uuid, d.bdf, d.gfx,
             (double)d.vram_total / (1ull << 30), d.numa_node, d.render_minor, d.compute_partition,
             d.memory_partition, d.name);
    }
    if (n > 1) {
      printf("links:\n     ");
      for (int j = 0; j < n; ++j) printf(" GPU%-3d", j);
      printf("\n");
      for (int i = 0; i < n; ++i) {
        printf("GPU%-2d", i);
        for (int j = 0; j < n; ++j) {
          gs_link_t L;
          gs_get_link(h, i, j, &L);
          printf(" %-4s%d ", link_name(L.type), L.hops);
        }
        printf("\n");
      }
    }
  }
  if (events_s > 0) {
    gs_events_start(h);
    for (int t = 0; t < events_s * 10; ++t) {
      gs_event_t ev;
      if (gs_wait_event(h, 100, &ev) == 1) printf("event dev=%d kind=%d msg=%s\n", ev.index, ev.kind, ev.message);
    }
  }
  gs_close(h);
  return 0;
}
