/*
 * lab3 stdin-grammar probe (reference lab3/src/test_read_input.c): parses the
 * class block "<nc>\n<np x y ...>\n..." and echoes it, so a hand-written input
 * can be checked before it is fed to the classifier. Also validates counts.
 */
#include <stdio.h>
#include <stdlib.h>

int main(void) {
    int nc;
    if (scanf("%d", &nc) != 1 || nc < 1) {
        fprintf(stderr, "expected a positive class count\n");
        return 1;
    }
    for (int c = 0; c < nc; ++c) {
        int np;
        if (scanf("%d", &np) != 1 || np < 1) {
            fprintf(stderr, "class %d: expected a positive point count\n", c + 1);
            return 1;
        }
        int *xy = (int *)malloc(sizeof(int) * 2 * (size_t)np);
        if (!xy) return 1;
        for (int i = 0; i < 2 * np; ++i)
            if (scanf("%d", &xy[i]) != 1) {
                fprintf(stderr, "class %d: truncated coordinates\n", c + 1);
                free(xy);
                return 1;
            }
        printf("Class %d:\n", c + 1);
        printf("Pixel count: %d\n", np);
        printf("Coordinates:\n");
        for (int i = 0; i < np; ++i) printf("(%d, %d)\n", xy[2 * i], xy[2 * i + 1]);
        free(xy);
    }
    return 0;
}
