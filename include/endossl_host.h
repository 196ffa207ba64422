/* endossl_host.h -- C-ABI of libendossl_host.so: the host-side input path of the SSL trainers.
 *
 * Replaces the reference's DataLoader-worker transforms (torchvision on PIL images):
 *   TransformFixMatch            code/dataset.py:24-56     (weak / strong views; also SemiFormer's)
 *   TransformCoMatch             code/dataset.py:58-110    (weak / strong_0 / strong_1 views)
 *   the labeled train transform  code/dataset.py:185-207   (without ToTensor/Normalize)
 *   the evaluation transform     code/dataset.py:217-231   (Resize -> CenterCrop)
 *   RandAugmentMC + its pool     code/randaugment.py:20-163,207-222
 * ToTensor + Normalize (code/dataset.py:49-51) are NOT here: the device applies them inside the patch
 * gather (es_patch_im2col_u8, include/endossl.h), so batches stay uint8 [n][3][S][S] end to end.
 *
 * Images are RGB, HWC, 3 bytes per pixel, rows contiguous.  Every op is bit-exact against PIL's
 * (tests/test_host_aug.py).  Status codes: 0 ok, 2 bad argument, 3 bad shape.  Thread-safe (no state). */
#ifndef ENDOSSL_HOST_H
#define ENDOSSL_HOST_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int esh_abi_version(void);

/* One pool op of fixmatch_augment_pool() (code/randaugment.py:147-163; index in that order:
 * AutoContrast, Brightness, Color, Contrast, Equalize, Identity, Posterize, Rotate, Sharpness, ShearX,
 * ShearY, Solarize, TranslateX, TranslateY) at magnitude v in [0, 10] (code/randaugment.py:139-144);
 * neg = the op's own `random.random() < 0.5` sign draw (Rotate / Shear / Translate).  src may be dst. */
int esh_aug_op(int op, const uint8_t* src, uint8_t* dst, int w, int h, int v, int neg);

/* ImageEnhance.{Brightness, Color, Contrast, Sharpness}(img).enhance(factor): kind 0..3
 * (code/randaugment.py:24-36,87-89; torchvision ColorJitter's brightness / contrast / saturation). */
int esh_enhance(int kind, const uint8_t* src, uint8_t* dst, int w, int h, float factor);

/* ColorJitter's hue (torchvision adjust_hue on a PIL image: HSV, hue += int8(factor * 255) mod 256,
 * back to RGB; factor in [-0.5, 0.5]) as kind 0, RandomGrayscale's 3-channel gray as kind 1
 * (code/dataset.py:76-79). */
int esh_color_op(int kind, const uint8_t* src, uint8_t* dst, int w, int h, double factor);

/* Image.rotate(angle_deg), NEAREST, no expand, fill 0 (code/randaugment.py:80-84; RandomRotation). */
int esh_rotate(const uint8_t* src, uint8_t* dst, int w, int h, double angle_deg);

/* Image.resize((ow, oh), BILINEAR) (torchvision Resize on a PIL image, code/dataset.py:28,32). */
int esh_resize_bilinear(const uint8_t* src, int w, int h, uint8_t* dst, int ow, int oh);

/* ImageDraw.rectangle((x0, y0, x1, y1), (v, v, v)) in place, inclusive corners (CutoutAbs,
 * code/randaugment.py:47-60). */
int esh_fill_rect(uint8_t* img, int w, int h, int x0, int y0, int x1, int y1, int v);

/* RandomCrop(S, padding=pad, padding_mode='reflect') at offset (top, left) of the padded image
 * (code/dataset.py:35-37); dst [S][S][3]. */
int esh_pad_reflect_crop(const uint8_t* src, int w, int h, int pad, int top, int left, int S, uint8_t* dst);

/* Batch builder on nthreads host threads; image i's randomness keyed on (seed, i) only, so the result
 * does not depend on nthreads.  Outputs planar uint8 [n][3][S][S] (es_patch_im2col_u8's input).
 *   kind 0: TransformFixMatch -> out0 = weak, out1 = strong                    (code/dataset.py:24-56)
 *   kind 1: labeled train transform -> out0                                    (code/dataset.py:185-207)
 *   kind 2: TransformCoMatch -> out0 = weak, out1 = strong_0, out2 = strong_1  (code/dataset.py:58-110)
 *   kind 3: evaluation transform -> out0                                       (code/dataset.py:217-231)
 * is_crop: config.DATA.IS_CROP (Resize to int(1.2 S), then CenterCrop(S)); unused outputs may be NULL. */
int esh_transform_batch(int kind, const uint8_t* const* srcs, const int* ws, const int* hs, int n, int S,
                        int is_crop, uint64_t seed, int nthreads, uint8_t* out0, uint8_t* out1, uint8_t* out2);

#ifdef __cplusplus
}
#endif
#endif /* ENDOSSL_HOST_H */
