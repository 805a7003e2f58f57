// bre_pbrt_main.cpp — `bre_pbrt scene.pbrt`: the pbrt command line for scenes whose Integrator
// is "photonbeam" (src/main/pbrt.cpp: parse, WorldEnd -> Render, film written by the integrator),
// with the render on an MI355X.  Options: --quick, --outfile FILE, --device N (pbrt's --nthreads
// is accepted and ignored).  Exit status 0 on success.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/bre_pbrt.h"

int main(int argc, char **argv) {
    const char *scene = nullptr, *outfile = nullptr;
    int quick = 0, device = 0;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--quick")) quick = 1;
        else if (!strcmp(argv[i], "--outfile") && i + 1 < argc) outfile = argv[++i];
        else if (!strcmp(argv[i], "--device") && i + 1 < argc) device = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--nthreads") && i + 1 < argc) ++i;
        else if (argv[i][0] == '-') {
            fprintf(stderr, "usage: bre_pbrt [--quick] [--outfile file.pfm] [--device n] scene.pbrt\n");
            return 2;
        } else scene = argv[i];
    }
    if (!scene) {
        fprintf(stderr, "usage: bre_pbrt [--quick] [--outfile file.pfm] [--device n] scene.pbrt\n");
        return 2;
    }
    bre_pbrt *p = nullptr;
    const bre_status st = bre_pbrt_parse_file(scene, &p);
    int ne = 0, nw = 0;
    fputs(bre_pbrt_messages(p, &ne, &nw), stderr);
    if (st != BRE_OK) {
        bre_pbrt_free(p);
        return 1;
    }
    int32_t w = 0, h = 0;
    char fn[1024];
    bre_pbrt_get_film(p, &w, &h, nullptr, fn, sizeof(fn));
    const auto t0 = std::chrono::steady_clock::now();
    const bre_status rs = bre_pbrt_render(p, device, quick, outfile, 1, nullptr);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    bre_pbrt_free(p);
    if (rs != BRE_OK) {
        fprintf(stderr, "Error: render failed (status %d)\n", (int)rs);
        return 1;
    }
    printf("rendered %dx%d in %.3f s -> %s\n", w, h, s, outfile ? outfile : fn);
    return 0;
}
