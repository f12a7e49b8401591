/* HDF5 fixtures for the cooler file boundary, written
 * by the real libhdf5 (1.10.6 in /opt/conda of the build container; compile
 * with `h5cc -O2 -o make_h5_fixtures make_h5_fixtures.c`, see
 * tests/golden/make_h5_fixtures.sh).  Test infrastructure only.
 *
 *   make_h5_fixtures gen <dir>   write cooler_earliest.cool (libhdf5's default
 *                                "earliest" format bounds, what h5py writes by
 *                                default) and cooler_latest.cool (libver latest:
 *                                superblock v3, v2 object headers, link
 *                                messages, dense attribute storage, fixed /
 *                                extensible array and single-chunk indexes)
 *   make_h5_fixtures dump <file> print a canonical listing of every group,
 *                                dataset (type, shape, layout, filters, values)
 *                                and attribute, as read back by libhdf5
 *
 * The files follow the layout cooler's create_cooler / `cooler balance`
 * produce through h5py for HiCHap's `file::res` URIs
 * (/root/reference/HiCHap/matrixBuilding.py:200-205, :708): one group per
 * resolution with chroms/{name (fixed-length NUL-padded ASCII), length},
 * bins/{chrom (enum over the chromosome names), start, end, weight},
 * pixels/{bin1_id, bin2_id, count}, indexes/{chrom_offset, bin1_offset};
 * every table chunked with shuffle + gzip-6 (bins/weight: gzip-6 only, as
 * `cooler balance` stores it); the info attributes as variable-length UTF-8
 * strings and int64 scalars; balance attributes with h5py's bool enum.  The
 * contents are synthetic and deterministic (an LCG), not HiCHap output. */
#include <hdf5.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHECK(x) do { if ((x) < 0) { fprintf(stderr, "HDF5 call failed at line %d\n", __LINE__); exit(2); } } while (0)

static uint64_t lcg_state = 20201015u;
static uint32_t lcg(void) {
    lcg_state = lcg_state * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(lcg_state >> 33);
}

/* ---------------------------------------------------------------- writing */
static hid_t dcpl_chunked(hsize_t chunk, int shuffle, int gzip) {
    hid_t p = H5Pcreate(H5P_DATASET_CREATE);
    CHECK(H5Pset_chunk(p, 1, &chunk));
    if (shuffle) CHECK(H5Pset_shuffle(p));
    if (gzip) CHECK(H5Pset_deflate(p, 6));
    return p;
}

static void write_1d(hid_t g, const char* name, hid_t ftype, hid_t mtype, const void* data, hsize_t n,
                     hsize_t chunk, int shuffle, int gzip, int unlimited) {
    hsize_t maxd = unlimited ? H5S_UNLIMITED : n;
    hid_t sp = H5Screate_simple(1, &n, &maxd);
    if (chunk > n && !unlimited) chunk = n > 0 ? n : 1;
    hid_t dcpl = dcpl_chunked(chunk, shuffle, gzip);
    hid_t d = H5Dcreate2(g, name, ftype, sp, H5P_DEFAULT, dcpl, H5P_DEFAULT);
    CHECK(d);
    if (n) CHECK(H5Dwrite(d, mtype, H5S_ALL, H5S_ALL, H5P_DEFAULT, data));
    H5Dclose(d);
    H5Pclose(dcpl);
    H5Sclose(sp);
}

static hid_t vlen_utf8(void) {
    hid_t t = H5Tcopy(H5T_C_S1);
    CHECK(H5Tset_size(t, H5T_VARIABLE));
    CHECK(H5Tset_cset(t, H5T_CSET_UTF8));
    return t;
}

static void attr_str(hid_t obj, const char* name, const char* v) {
    hid_t t = vlen_utf8();
    hid_t sp = H5Screate(H5S_SCALAR);
    hid_t a = H5Acreate2(obj, name, t, sp, H5P_DEFAULT, H5P_DEFAULT);
    CHECK(a);
    CHECK(H5Awrite(a, t, &v));
    H5Aclose(a);
    H5Sclose(sp);
    H5Tclose(t);
}

static void attr_i64(hid_t obj, const char* name, int64_t v) {
    hid_t sp = H5Screate(H5S_SCALAR);
    hid_t a = H5Acreate2(obj, name, H5T_STD_I64LE, sp, H5P_DEFAULT, H5P_DEFAULT);
    CHECK(a);
    CHECK(H5Awrite(a, H5T_NATIVE_INT64, &v));
    H5Aclose(a);
    H5Sclose(sp);
}

static void attr_f64(hid_t obj, const char* name, const double* v, int n) {
    hsize_t d = (hsize_t)n;
    hid_t sp = n ? H5Screate_simple(1, &d, NULL) : H5Screate(H5S_SCALAR);
    hid_t a = H5Acreate2(obj, name, H5T_IEEE_F64LE, sp, H5P_DEFAULT, H5P_DEFAULT);
    CHECK(a);
    CHECK(H5Awrite(a, H5T_NATIVE_DOUBLE, v));
    H5Aclose(a);
    H5Sclose(sp);
}

static hid_t bool_enum(void) { /* h5py's numpy bool: enum over int8 {FALSE, TRUE} */
    hid_t t = H5Tenum_create(H5T_NATIVE_INT8);
    int8_t f = 0, tr = 1;
    CHECK(H5Tenum_insert(t, "FALSE", &f));
    CHECK(H5Tenum_insert(t, "TRUE", &tr));
    return t;
}

static void attr_bool(hid_t obj, const char* name, const int8_t* v, int n) {
    hsize_t d = (hsize_t)n;
    hid_t t = bool_enum();
    hid_t sp = n ? H5Screate_simple(1, &d, NULL) : H5Screate(H5S_SCALAR);
    hid_t a = H5Acreate2(obj, name, t, sp, H5P_DEFAULT, H5P_DEFAULT);
    CHECK(a);
    CHECK(H5Awrite(a, t, v));
    H5Aclose(a);
    H5Sclose(sp);
    H5Tclose(t);
}

typedef struct {
    const char* name;
    int32_t length;
} chrom_t;

static const chrom_t CHROMS[] = {{"chr1", 2000000}, {"chr22", 1500000}, {"chrX", 900000}};
#define NCHROMS 3

static void write_resolution(hid_t file, int32_t res, int latest, int cis_only_weight) {
    char gname[32];
    snprintf(gname, sizeof gname, "%d", res);
    hid_t g = H5Gcreate2(file, gname, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    CHECK(g);
    /* bins: the reference's l // res + 1 per chromosome (matrixBuilding.py:564) is
     * HiCHap's own dense layout; cooler's binnify gives ceil(l / res) */
    int32_t nb_chrom[NCHROMS];
    int64_t nbins = 0;
    for (int c = 0; c < NCHROMS; ++c) {
        nb_chrom[c] = (CHROMS[c].length + res - 1) / res;
        nbins += nb_chrom[c];
    }
    int32_t* bchrom = malloc(sizeof(int32_t) * nbins);
    int32_t* bstart = malloc(sizeof(int32_t) * nbins);
    int32_t* bend = malloc(sizeof(int32_t) * nbins);
    int64_t* chrom_offset = malloc(sizeof(int64_t) * (NCHROMS + 1));
    int64_t k = 0;
    for (int c = 0; c < NCHROMS; ++c) {
        chrom_offset[c] = k;
        for (int32_t i = 0; i < nb_chrom[c]; ++i, ++k) {
            bchrom[k] = c;
            bstart[k] = i * res;
            bend[k] = (i + 1) * res < CHROMS[c].length ? (i + 1) * res : CHROMS[c].length;
        }
    }
    chrom_offset[NCHROMS] = nbins;
    /* pixels: upper triangle, sorted by (bin1, bin2); decaying cis + sparse trans */
    int64_t cap = nbins * nbins, npx = 0;
    int64_t* b1 = malloc(sizeof(int64_t) * cap);
    int64_t* b2 = malloc(sizeof(int64_t) * cap);
    int32_t* cnt = malloc(sizeof(int32_t) * cap);
    int64_t* bin1_offset = malloc(sizeof(int64_t) * (nbins + 1));
    for (int64_t i = 0; i < nbins; ++i) {
        bin1_offset[i] = npx;
        for (int64_t j = i; j < nbins; ++j) {
            const int cis = bchrom[i] == bchrom[j];
            const int64_t d = j - i;
            const uint32_t r = lcg() % 1000;
            int keep = cis ? (d < 4 || r < 600 / (d + 1) + 20) : r < 8;
            if (!keep) continue;
            b1[npx] = i;
            b2[npx] = j;
            cnt[npx] = cis ? (int32_t)(1 + (lcg() % (4000 / (d + 1) + 3))) : (int32_t)(1 + lcg() % 3);
            if (lcg() % 97 == 0) cnt[npx] += 70000; /* a few counts beyond uint16 */
            ++npx;
        }
    }
    bin1_offset[nbins] = npx;

    hid_t gc = H5Gcreate2(g, "chroms", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    char names[NCHROMS][5];
    int32_t lengths[NCHROMS];
    memset(names, 0, sizeof names);
    for (int c = 0; c < NCHROMS; ++c) {
        memcpy(names[c], CHROMS[c].name, strlen(CHROMS[c].name));
        lengths[c] = CHROMS[c].length;
    }
    hid_t st = H5Tcopy(H5T_C_S1); /* numpy 'S5': fixed length, NUL-padded, ASCII */
    CHECK(H5Tset_size(st, 5));
    CHECK(H5Tset_strpad(st, H5T_STR_NULLPAD));
    write_1d(gc, "name", st, st, names, NCHROMS, NCHROMS, 1, 1, 0);
    H5Tclose(st);
    write_1d(gc, "length", H5T_STD_I32LE, H5T_NATIVE_INT32, lengths, NCHROMS, NCHROMS, 1, 1, 0);
    H5Gclose(gc);

    hid_t gb = H5Gcreate2(g, "bins", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    hid_t en = H5Tenum_create(H5T_STD_I32LE);
    for (int c = 0; c < NCHROMS; ++c) CHECK(H5Tenum_insert(en, CHROMS[c].name, &c));
    hid_t enm = H5Tenum_create(H5T_NATIVE_INT32);
    for (int c = 0; c < NCHROMS; ++c) CHECK(H5Tenum_insert(enm, CHROMS[c].name, &c));
    const hsize_t bchunk = nbins > 40 ? 40 : (hsize_t)nbins; /* several chunks, a ragged last one */
    write_1d(gb, "chrom", en, enm, bchrom, nbins, bchunk, 1, 1, 0);
    H5Tclose(en);
    H5Tclose(enm);
    write_1d(gb, "start", H5T_STD_I32LE, H5T_NATIVE_INT32, bstart, nbins, bchunk, 1, 1, 0);
    write_1d(gb, "end", H5T_STD_I32LE, H5T_NATIVE_INT32, bend, nbins, bchunk, 1, 1, 0);
    { /* bins/weight as `cooler balance` writes it (gzip 6, no shuffle) */
        double* w = malloc(sizeof(double) * nbins);
        for (int64_t i = 0; i < nbins; ++i)
            w[i] = (i % 17 == 5) ? (0.0 / 0.0) : 1.0 / (1.0 + (double)(lcg() % 100000) / 7919.0);
        hsize_t n = (hsize_t)nbins;
        hid_t sp = H5Screate_simple(1, &n, NULL);
        hid_t dcpl = dcpl_chunked(n, 0, 1);
        hid_t d = H5Dcreate2(gb, "weight", H5T_IEEE_F64LE, sp, H5P_DEFAULT, dcpl, H5P_DEFAULT);
        CHECK(d);
        CHECK(H5Dwrite(d, H5T_NATIVE_DOUBLE, H5S_ALL, H5S_ALL, H5P_DEFAULT, w));
        double tol = 1e-5;
        attr_f64(d, "tol", &tol, 0);
        attr_i64(d, "min_nnz", 10);
        attr_i64(d, "min_count", 0);
        attr_i64(d, "mad_max", 5);
        int8_t co = (int8_t)cis_only_weight, dw = 0;
        attr_bool(d, "cis_only", &co, 0);
        attr_i64(d, "ignore_diags", 1);
        if (cis_only_weight) {
            double sc[NCHROMS] = {101.5, 87.25, 40.125}, var[NCHROMS] = {3e-6, 8.5e-6, 1e-7};
            int8_t cv[NCHROMS] = {1, 1, 0};
            attr_f64(d, "scale", sc, NCHROMS);
            attr_bool(d, "converged", cv, NCHROMS);
            attr_f64(d, "var", var, NCHROMS);
        } else {
            double sc = 1234.5678, var = 9.5e-6;
            int8_t cv = 1;
            attr_f64(d, "scale", &sc, 0);
            attr_bool(d, "converged", &cv, 0);
            attr_f64(d, "var", &var, 0);
        }
        attr_bool(d, "divisive_weights", &dw, 0);
        H5Dclose(d);
        H5Pclose(dcpl);
        H5Sclose(sp);
        free(w);
    }
    H5Gclose(gb);

    hid_t gp = H5Gcreate2(g, "pixels", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    /* resizable tables (cooler appends pixel chunks): unlimited max shape;
     * small chunks so the earliest-format chunk B-tree has two levels */
    write_1d(gp, "bin1_id", H5T_STD_I64LE, H5T_NATIVE_INT64, b1, npx, 8, 1, 1, 1);
    write_1d(gp, "bin2_id", H5T_STD_I64LE, H5T_NATIVE_INT64, b2, npx, 8, 1, 1, 1);
    write_1d(gp, "count", H5T_STD_I32LE, H5T_NATIVE_INT32, cnt, npx, 20, 1, 1, 1);
    H5Gclose(gp);

    hid_t gi = H5Gcreate2(g, "indexes", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    write_1d(gi, "chrom_offset", H5T_STD_I64LE, H5T_NATIVE_INT64, chrom_offset, NCHROMS + 1, NCHROMS + 1, 1, 1, 0);
    write_1d(gi, "bin1_offset", H5T_STD_I64LE, H5T_NATIVE_INT64, bin1_offset, nbins + 1, 64, 1, 1, 0);
    H5Gclose(gi);

    /* cooler's info attributes on the resolution group (cooler/_create.py write_info) */
    attr_str(g, "format", "HDF5::Cooler");
    attr_i64(g, "format-version", 3);
    attr_str(g, "format-url", "https://github.com/mirnylab/cooler");
    attr_str(g, "generated-by", "make_h5_fixtures.c (cooler schema v3)");
    attr_str(g, "creation-date", "2020-10-15T00:00:00.000000");
    attr_str(g, "bin-type", "fixed");
    attr_i64(g, "bin-size", res);
    attr_str(g, "storage-mode", "symmetric-upper");
    attr_i64(g, "nbins", nbins);
    attr_i64(g, "nchroms", NCHROMS);
    attr_i64(g, "nnz", npx);
    attr_str(g, "metadata", latest ? "{\"format\": \"latest\", \"note\": \"\xc3\xa9t\xc3\xa9\"}" : "{}");
    attr_str(g, "assembly", "hg19");
    H5Gclose(g);
    (void)latest;
    free(bchrom); free(bstart); free(bend); free(chrom_offset);
    free(b1); free(b2); free(cnt); free(bin1_offset);
}

static void gen(const char* dir, int latest) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s", dir, latest ? "cooler_latest.cool" : "cooler_earliest.cool");
    hid_t fapl = H5Pcreate(H5P_FILE_ACCESS);
    if (latest) CHECK(H5Pset_libver_bounds(fapl, H5F_LIBVER_LATEST, H5F_LIBVER_LATEST));
    hid_t f = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, fapl);
    CHECK(f);
    lcg_state = latest ? 7u : 20201015u;
    write_resolution(f, 40000, latest, 0);
    write_resolution(f, 500000, latest, 1);
    /* more resolutions in the latest-format file: a root group of more than 8
     * links is stored densely (fractal heap + v2 B-tree name index) */
    if (latest)
        for (int r = 1; r <= 8; ++r) write_resolution(f, 600000 + 100000 * r, latest, r & 1);
    H5Fclose(f);
    H5Pclose(fapl);
}

/* ---------------------------------------------------------------- dumping */
static void hex(const unsigned char* p, size_t n) {
    for (size_t i = 0; i < n; ++i) printf("%02x", p[i]);
}

/* type tag: i<n>/u<n> (little endian), f<n>, S<n>, vstr, enum(<base>){name=value,...} */
static void type_tag(hid_t t) {
    H5T_class_t c = H5Tget_class(t);
    size_t sz = H5Tget_size(t);
    if (c == H5T_INTEGER) {
        printf("%c%zu", H5Tget_sign(t) == H5T_SGN_NONE ? 'u' : 'i', sz);
    } else if (c == H5T_FLOAT) {
        printf("f%zu", sz);
    } else if (c == H5T_STRING) {
        if (H5Tis_variable_str(t) > 0) printf("vstr");
        else printf("S%zu", sz);
    } else if (c == H5T_ENUM) {
        hid_t b = H5Tget_super(t);
        printf("enum(");
        type_tag(b);
        printf("){");
        int nm = H5Tget_nmembers(t);
        for (int i = 0; i < nm; ++i) {
            char* name = H5Tget_member_name(t, (unsigned)i);
            long long v = 0;
            CHECK(H5Tget_member_value(t, (unsigned)i, &v)); /* little-endian host: low bytes */
            if (H5Tget_size(b) == 1) v = (signed char)v;
            else if (H5Tget_size(b) == 2) v = (short)v;
            else if (H5Tget_size(b) == 4) v = (int)v;
            printf("%s%s=%lld", i ? "," : "", name, v);
            H5free_memory(name);
        }
        printf("}");
        H5Tclose(b);
    } else {
        printf("class%d", (int)c);
    }
}

/* values: integers in decimal, floats as their IEEE bit patterns in hex,
 * strings as the hex of their bytes (fixed: the whole padded field) */
static void one_value(hid_t t, const unsigned char* p) {
    H5T_class_t c = H5Tget_class(t);
    size_t sz = H5Tget_size(t);
    {
        if (c == H5T_ENUM) {
            hid_t b = H5Tget_super(t);
            one_value(b, p);
            H5Tclose(b);
            return;
        }
        if (c == H5T_INTEGER) {
            const int s = H5Tget_sign(t) != H5T_SGN_NONE;
            if (sz == 1) printf("%lld", s ? (long long)*(const int8_t*)p : (long long)*(const uint8_t*)p);
            else if (sz == 2) printf("%lld", s ? (long long)*(const int16_t*)p : (long long)*(const uint16_t*)p);
            else if (sz == 4) printf("%lld", s ? (long long)*(const int32_t*)p : (long long)*(const uint32_t*)p);
            else if (s) printf("%lld", (long long)*(const int64_t*)p);
            else printf("%llu", (unsigned long long)*(const uint64_t*)p);
        } else if (c == H5T_FLOAT) {
            if (sz == 8) printf("%016" PRIx64, *(const uint64_t*)p);
            else printf("%08" PRIx32, *(const uint32_t*)p);
        } else if (c == H5T_STRING && H5Tis_variable_str(t) > 0) {
            const char* s = *(const char* const*)p;
            putchar('x');
            if (s) hex((const unsigned char*)s, strlen(s));
        } else {
            putchar('x');
            hex(p, sz);
        }
    }
}

static void values(hid_t t, const unsigned char* buf, size_t n) {
    const size_t sz = H5Tget_size(t);
    for (size_t i = 0; i < n; ++i) {
        putchar(' ');
        one_value(t, buf + i * sz);
    }
}

static void shape_of(hid_t sp, hsize_t* n) {
    int r = H5Sget_simple_extent_ndims(sp);
    hsize_t d[8];
    H5Sget_simple_extent_dims(sp, d, NULL);
    *n = 1;
    printf(" shape=(");
    for (int i = 0; i < r; ++i) {
        printf("%s%llu", i ? "," : "", (unsigned long long)d[i]);
        *n *= d[i];
    }
    printf(")");
}

static herr_t dump_attr(hid_t obj, const char* name, const H5A_info_t* info, void* opdata) {
    (void)info;
    const char* path = (const char*)opdata;
    hid_t a = H5Aopen(obj, name, H5P_DEFAULT);
    hid_t t = H5Aget_type(a), sp = H5Aget_space(a);
    hid_t mt = H5Tget_class(t) == H5T_STRING && H5Tis_variable_str(t) > 0 ? H5Tcopy(t) : H5Tget_native_type(t, H5T_DIR_ASCEND);
    printf("A %s@%s ", path, name);
    type_tag(t);
    hsize_t n;
    shape_of(sp, &n);
    size_t sz = H5Tget_size(mt);
    unsigned char* buf = calloc(n ? n : 1, sz);
    CHECK(H5Aread(a, mt, buf));
    printf(" =");
    values(mt, buf, n);
    printf("\n");
    if (H5Tget_class(t) == H5T_STRING && H5Tis_variable_str(t) > 0) H5Dvlen_reclaim(mt, sp, H5P_DEFAULT, buf);
    free(buf);
    H5Tclose(mt); H5Tclose(t); H5Sclose(sp); H5Aclose(a);
    return 0;
}

static herr_t visit(hid_t root, const char* name, const H5O_info_t* info, void* op) {
    (void)op;
    char path[1024];
    if (strcmp(name, ".") == 0) snprintf(path, sizeof path, "/");
    else snprintf(path, sizeof path, "/%s", name);
    hid_t o = H5Oopen(root, name, H5P_DEFAULT);
    if (info->type == H5O_TYPE_GROUP) {
        printf("G %s\n", path);
    } else if (info->type == H5O_TYPE_DATASET) {
        hid_t t = H5Dget_type(o), sp = H5Dget_space(o), dcpl = H5Dget_create_plist(o);
        hid_t mt = H5Tget_class(t) == H5T_STRING && H5Tis_variable_str(t) > 0 ? H5Tcopy(t) : H5Tget_native_type(t, H5T_DIR_ASCEND);
        printf("D %s ", path);
        type_tag(t);
        hsize_t n;
        shape_of(sp, &n);
        H5D_layout_t lay = H5Pget_layout(dcpl);
        if (lay == H5D_CHUNKED) {
            hsize_t c[8];
            int r = H5Pget_chunk(dcpl, 8, c);
            printf(" chunked(");
            for (int i = 0; i < r; ++i) printf("%s%llu", i ? "," : "", (unsigned long long)c[i]);
            printf(")");
        } else {
            printf(" %s", lay == H5D_CONTIGUOUS ? "contiguous" : "compact");
        }
        int nf = H5Pget_nfilters(dcpl);
        printf(" filters=[");
        for (int i = 0; i < nf; ++i) {
            unsigned flags, cd[8];
            size_t ncd = 8;
            H5Z_filter_t id = H5Pget_filter2(dcpl, (unsigned)i, &flags, &ncd, cd, 0, NULL, NULL);
            printf("%s%d", i ? "," : "", (int)id);
        }
        printf("]\n");
        size_t sz = H5Tget_size(mt);
        unsigned char* buf = calloc(n ? n : 1, sz);
        if (n) CHECK(H5Dread(o, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, buf));
        printf("V %s =", path);
        values(mt, buf, n);
        printf("\n");
        free(buf);
        H5Tclose(mt); H5Tclose(t); H5Sclose(sp); H5Pclose(dcpl);
    }
    H5Aiterate2(o, H5_INDEX_NAME, H5_ITER_INC, NULL, dump_attr, path);
    H5Oclose(o);
    return 0;
}

static int dump(const char* path) {
    hid_t f = H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
    if (f < 0) return 3;
    CHECK(H5Ovisit(f, H5_INDEX_NAME, H5_ITER_INC, visit, NULL));
    H5Fclose(f);
    return 0;
}

int main(int argc, char** argv) {
    if (argc == 3 && strcmp(argv[1], "gen") == 0) {
        gen(argv[2], 0);
        gen(argv[2], 1);
        return 0;
    }
    if (argc == 3 && strcmp(argv[1], "dump") == 0) return dump(argv[2]);
    fprintf(stderr, "usage: %s gen <dir> | dump <file>\n", argv[0]);
    return 1;
}
