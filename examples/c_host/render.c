/* render.c — a plain C host driving the trace path through the C-ABI only
 * (include/rt_trace.h), the way the reference's platform layer drives
 * OnInit / OnRender (wasm/wasm.cpp, win32/win32.cpp -> main.cpp:645-859).
 *
 * usage: render <width> <height> <frames> <scene> <out-prefix> [hip-devices, e.g. 0 or 0,0,0]
 *
 * One OnRender call per progressive frame with the reference's one-frame
 * output lag: the first call starts frame 0 and returns no image, each later
 * call returns the previous completed frame.  Every completed frame k is
 * written as raw RGBA8 (<out-prefix>.<k>.rgba, row 0 first) and the last one
 * also as a PNG; one line per frame reports the ray count.  With more than one
 * device the frames are traced in bands across them (rt_on_init_devices). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_trace.h"

static int die(const char *what, int rc) {
    fprintf(stderr, "render: %s failed (%d): %s\n", what, rc, rt_last_error());
    return 1;
}

static int parse_devices(const char *s, int *out, uint32_t cap) {
    uint32_t n = 0;
    while (*s && n < cap) {
        char *end = NULL;
        long v = strtol(s, &end, 10);
        if (end == s || v < 0) return -1;
        out[n++] = (int)v;
        s = *end == ',' ? end + 1 : end;
    }
    return (int)n;
}

int main(int argc, char **argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s <width> <height> <frames> <scene> <out-prefix> [devices]\n", argv[0]);
        return 2;
    }
    const uint32_t W = (uint32_t)atoi(argv[1]), H = (uint32_t)atoi(argv[2]);
    const uint32_t frames = (uint32_t)atoi(argv[3]), scene = (uint32_t)atoi(argv[4]);
    const char *prefix = argv[5];
    int devices[RT_MULTI_MAX_DEVICES] = {0};
    int n_dev = argc > 6 ? parse_devices(argv[6], devices, RT_MULTI_MAX_DEVICES) : 1;
    if (W == 0 || H == 0 || frames == 0 || n_dev <= 0) {
        fprintf(stderr, "render: bad arguments\n");
        return 2;
    }

    rt_init_params init = {W, H, "render", 6};
    int rc = n_dev > 1 ? rt_on_init_devices(&init, devices, (uint32_t)n_dev) : rt_on_init(&init);
    if (rc != RT_OK) return die("rt_on_init", rc);

    uint32_t *pixels = (uint32_t *)calloc((size_t)W * H, sizeof(uint32_t));
    if (!pixels) return die("calloc", RT_ENOMEM);
    rt_image image = {pixels, W, H, RT_FORMAT_R8G8B8A8_U32};
    rt_render_params params = {1u, true, scene};

    uint64_t rays = 0;
    double ms = 0.0;
    rc = rt_on_render(&image, params, 0u, &rays, &ms);  /* starts frame 0, no image yet */
    if (rc < 0) return die("rt_on_render", rc);
    if (rc != 0) {
        fprintf(stderr, "render: the first OnRender call returned a frame\n");
        return 1;
    }
    for (uint32_t k = 0; k < frames; ++k) {
        if ((rc = rt_on_render_wait()) != RT_OK) return die("rt_on_render_wait", rc);
        rc = rt_on_render(&image, params, 0u, &rays, &ms);
        if (rc < 0) return die("rt_on_render", rc);
        if (rc != 1) {
            fprintf(stderr, "render: frame %u did not complete\n", k);
            return 1;
        }
        char path[1024];
        snprintf(path, sizeof(path), "%s.%u.rgba", prefix, k);
        FILE *f = fopen(path, "wb");
        if (!f || fwrite(pixels, sizeof(uint32_t), (size_t)W * H, f) != (size_t)W * H) return die(path, RT_EIO);
        fclose(f);
        printf("frame %u rays %llu ms %.3f\n", k, (unsigned long long)rays, ms);
    }
    if ((rc = rt_on_render_wait()) != RT_OK) return die("rt_on_render_wait", rc);
    char png[1024];
    snprintf(png, sizeof(png), "%s.png", prefix);
    if ((rc = rt_image_write_png(&image, png, RT_IMAGE_FLIP_Y)) != RT_OK) return die("rt_image_write_png", rc);
    if ((rc = rt_on_shutdown()) != RT_OK) return die("rt_on_shutdown", rc);
    free(pixels);
    return 0;
}
