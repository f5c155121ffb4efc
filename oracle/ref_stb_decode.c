/* TEST INFRASTRUCTURE ONLY — decodes image files with the reference's own
 * stb_image (external/stb/stb_image.h v2.30, compiled from /root/reference by
 * `make -C oracle ref`), exactly as Texture2D(path) does
 * (external/OpenGL/textureClass.cpp:55-68: stbi_set_flip_vertically_on_load(true),
 * stbi_load(path, &w, &h, &n, 0)).  Used only to make the golden fixtures the
 * product decoder is checked against (tests/golden/make_texture_golden.py).
 *
 *   ref_stb_decode <image> <out.raw>   ->  prints "w h n", writes w*h*n bytes
 */
#define STB_IMAGE_IMPLEMENTATION
#include "stb/stb_image.h"

#include <stdio.h>

int main(int argc, char** argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s <image> <out.raw>\n", argv[0]);
        return 2;
    }
    stbi_set_flip_vertically_on_load(1);
    int w = 0, h = 0, n = 0;
    unsigned char* px = stbi_load(argv[1], &w, &h, &n, 0);
    if (!px) {
        fprintf(stderr, "stbi_load failed: %s\n", stbi_failure_reason());
        return 1;
    }
    FILE* f = fopen(argv[2], "wb");
    if (!f) return 1;
    fwrite(px, 1, (size_t)w * h * n, f);
    fclose(f);
    stbi_image_free(px);
    printf("%d %d %d\n", w, h, n);
    return 0;
}
