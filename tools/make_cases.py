#!/usr/bin/env python3
"""Write tests/golden/cases.txt: the datatype zoo the golden vectors cover.

One line per case: ``name | count | recipe`` (recipe language: oracle/recipe.h).
The list follows SURVEY.md sec. 8(c): the reference's own parity matrix
(/root/reference/test/pack_unpack.cpp:155-297), its type factories
(/root/reference/support/type.cpp:3-308), the bench-mpi-pack type
(/root/reference/bin/bench_mpi_pack.cpp), halo-exchange face/edge/corner types
at a reduced grid (/root/reference/bin/bench_halo_exchange.cpp:87-168), small
2D/3D subarray sweeps, the F1/F2 witnesses, and edge cases (zero counts,
negative strides, resized, Fortran order, non-byte base types, the
constructors TEMPI must hand to the library).
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden", "cases.txt")


def vec3(copy, alloc):
    """make_byte_v_hv (support/type.cpp:66-89)."""
    cx, cy, cz = copy
    ax, ay, az = alloc
    return f"hvector({cz},1,{ax*ay},vector({cy},{cx},{ax},byte))"


def halo_type(radius, lcr, pitch, ysize, d, q, exterior):
    """halo_type (bench_halo_exchange.cpp:87-168): subarray of the padded block."""
    pos, ext = [], []
    for k in range(3):
        if d[k] == -1:
            pos.append(0 if exterior else radius)
        elif d[k] == 1:
            pos.append(lcr[k] + (radius if exterior else 0))
        else:
            pos.append(radius)
        ext.append(lcr[k] if d[k] == 0 else radius)
    sizes = [pos[2] + ext[2], ysize, pitch]
    subs = [ext[2], ext[1], ext[0] * q]
    starts = [pos[2], pos[1], pos[0] * q]
    return "subarray(C,[%s],[%s],[%s],byte)" % tuple(",".join(map(str, v)) for v in (sizes, subs, starts))


def cases():
    c = []
    add = lambda name, count, recipe: c.append((name, count, recipe))

    # --- reference parity matrix: test/pack_unpack.cpp:155-297
    add("ref_contiguous_contiguous_10", 30, "contig(10,byte)")
    for n in (1, 2):
        add(f"ref_2d_byte_vector_2_3_4_x{n}", n, "vector(2,3,4,byte)")
        add(f"ref_2d_byte_subarray_2_3_4_x{n}", n, "subarray(C,[2,4],[2,3],[0,0],byte)")
        add(f"ref_off_subarray_234_16c_114_x{n}", n, "subarray(C,[16,16,16],[2,3,4],[1,1,4],byte)")
    add("ref_byte_v_hv_234_10c_x1", 1, vec3((2, 3, 4), (10, 10, 10)))
    add("ref_byte_v_hv_234_10c_x2", 2, vec3((2, 3, 4), (10, 10, 10)))
    add("ref_byte_v_hv_10_10_1_10c_x1", 1, vec3((10, 10, 1), (10, 10, 10)))
    add("ref_byte_v_hv_434_200c_x1", 1, vec3((4, 3, 4), (200, 200, 200)))
    add("ref_byte_v_hv_100c_200c_x1", 1, vec3((100, 100, 100), (200, 200, 200)))
    add("ref_byte_v_hv_100c_200c_x3", 3, vec3((100, 100, 100), (200, 200, 200)))

    # --- bench-mpi-pack / config 1: MPI_Type_vector(1024, 512, 1024, MPI_BYTE)
    add("cfg1_vector_1024_512_1024", 1, "vector(1024,512,1024,byte)")
    add("cfg1_hvector_1024_512_1024", 1, "hvector(1024,512,1024,byte)")
    add("cfg1_subarray_1024_512_1024", 1, "subarray(C,[1024,1024],[1024,512],[0,0],byte)")

    # --- support/type.cpp factories (3D copy 5x3x4 of alloc 16x8x8, bytes)
    cp, al = (5, 3, 4), (16, 8, 8)
    add("zoo_byte_vn_hv_hv", 1, f"hvector({cp[2]},1,{al[0]*al[1]},hvector({cp[1]},1,{al[0]},vector({cp[0]},1,1,byte)))")
    add("zoo_byte_v1_hv_hv", 1, f"hvector({cp[2]},1,{al[0]*al[1]},hvector({cp[1]},1,{al[0]},vector(1,{cp[0]},{al[0]},byte)))")
    add("zoo_byte_v_hv", 2, vec3(cp, al))
    add("zoo_float_v_hv", 1, f"hvector(4,1,{32*8},vector(3,{8//4},{32//4},float))")
    rows = [(z * al[1] * al[0] + y * al[0]) for z in range(cp[2]) for y in range(cp[1])]
    add("zoo_hi", 1, "hindexed([%s],[%s],byte)" % (",".join([str(cp[0])] * len(rows)), ",".join(map(str, rows))))
    add("zoo_hib", 1, "hindexed_block(%d,[%s],byte)" % (cp[0], ",".join(map(str, rows))))
    add("zoo_subarray", 1, f"subarray(C,[{al[2]},{al[1]},{al[0]}],[{cp[2]},{cp[1]},{cp[0]}],[0,0,0],byte)")
    add("zoo_subarray_v", 1, f"vector({cp[2]},1,1,subarray(C,[{al[1]},{al[0]}],[{cp[1]},{cp[0]}],[0,0],byte))")
    add("zoo_2d_byte_hvector", 2, "hvector(7,5,12,byte)")
    add("zoo_contiguous_byte_v1", 3, "vector(37,1,1,byte)")
    add("zoo_contiguous_byte_vn", 3, "vector(1,37,37,byte)")
    add("zoo_contiguous_subarray", 3, "subarray(C,[37],[37],[0],byte)")
    add("zoo_contiguous_contiguous", 3, "contig(37,byte)")

    # --- SURVEY F1 witness: make_2d_hv_by_rows / _by_cols(13,3,16,5,53)
    add("f1_hv_by_rows", 1, "hvector(5,1,53,hvector(3,1,16,contig(13,byte)))")
    add("f1_hv_by_cols", 1, "hvector(3,1,16,hvector(5,1,53,contig(13,byte)))")
    add("f1_hv_by_cols_x2", 2, "hvector(3,1,16,hvector(5,1,53,contig(13,byte)))")
    # --- SURVEY F2 witness: 1D subarray keeps its extent
    add("f2_subarray1d_100_10_5", 3, "subarray(C,[100],[10],[5],byte)")
    add("f2_contig_resized_pad", 4, "resized(0,16,contig(10,byte))")

    # --- 2D subarray sweep (ragged block counts, strides 2*bl and bl+16)
    for bl in (1, 2, 3, 4, 8, 12, 16, 24, 64, 512):
        for stride in sorted({2 * bl, bl + 16}):
            nb = 37
            for n in (1, 2, 3):
                add(f"sweep2d_bl{bl}_st{stride}_x{n}", n, f"subarray(C,[{nb},{stride}],[{nb},{bl}],[0,0],byte)")
        # with a start offset on both axes
        add(f"sweep2d_off_bl{bl}", 2, f"subarray(C,[41,{2*bl+5}],[29,{bl}],[3,{bl//2+1}],byte)")

    # --- 3D subarray sweep
    for bl in (1, 3, 8, 24, 64, 200):
        add(f"sweep3d_bl{bl}_x1", 1, f"subarray(C,[9,7,{bl+13}],[5,4,{bl}],[2,1,6],byte)")
        add(f"sweep3d_bl{bl}_x2", 2, f"subarray(C,[9,7,{bl+13}],[5,4,{bl}],[2,1,6],byte)")

    # --- halo exchange types, 32^3 local region, radius 3, 8-byte quantities
    lcr, r, q = (32, 32, 32), 3, 8
    width = (lcr[0] + 2 * r) * q
    pitch = (width + 511) // 512 * 512
    ysize = lcr[1] + 2 * r
    for d in [(-1, 0, 0), (0, 1, 0), (0, 0, -1), (1, 1, 0), (0, -1, 1), (1, 1, 1), (-1, -1, -1)]:
        for exterior in (False, True):
            tag = "ext" if exterior else "int"
            add(f"halo32_{d[0]}_{d[1]}_{d[2]}_{tag}", 1, halo_type(r, lcr, pitch, ysize, d, q, exterior))

    # --- other base types / orders / markers
    add("float_vector", 2, "vector(9,3,5,float)")
    add("double_subarray_F", 1, "subarray(F,[7,6,5],[3,4,2],[1,2,3],double)")
    add("int_subarray_F_2d", 2, "subarray(F,[10,12],[4,5],[2,3],int)")
    add("double_hvector_of_vector", 1, "hvector(3,2,1000,vector(4,1,3,double))")
    add("vector_neg_stride", 2, "vector(4,3,-7,byte)")
    add("hvector_neg_stride", 1, "hvector(5,8,-40,byte)")
    add("resized_lb", 2, "resized(-4,48,vector(3,4,9,byte))")
    add("dup_vector", 2, "dup(vector(6,5,11,byte))")
    add("contig_of_vector", 2, "contig(3,vector(4,2,5,short))")
    add("vector_of_contig", 1, "vector(5,2,3,contig(4,int))")
    add("vector_count1", 2, "vector(1,17,40,byte)")
    add("vector_bl0", 1, "vector(4,0,5,byte)")
    add("count_zero", 0, "vector(4,3,5,byte)")
    add("subarray_sub1", 3, "subarray(C,[5,6,7],[1,6,7],[2,0,0],byte)")
    add("subarray_4d", 1, "subarray(C,[4,5,6,7],[2,3,4,5],[1,1,1,1],byte)")
    add("subarray_4d_x2", 2, "subarray(C,[4,5,6,7],[2,3,2,5],[1,1,3,1],byte)")
    add("indexed_regular", 1, "indexed([2,2,2,2],[0,5,10,15],int)")
    add("indexed_block_regular", 2, "indexed_block(3,[0,7,14],byte)")
    add("hindexed_irregular", 1, "hindexed([3,1,4],[0,9,20],byte)")
    # MPI_Type_create_struct with one element type (the reference refuses
    # every struct, src/internal/types.cpp:230; TEMPI folds these)
    add("struct_regular", 2, "struct([4,4,4,4],[0,24,48,72],short)")
    add("struct_of_vector", 1, "struct([1,1,1],[0,4000,8000],vector(30,3,10,byte))")
    add("struct_irregular", 1, "struct([2,5,1],[0,40,100],int)")
    add("struct_negative", 1, "struct([3,3],[64,-64],double)")
    add("nested_4level", 1, "hvector(2,1,5000,hvector(3,1,600,vector(4,5,30,byte)))")
    add("basic_double_x7", 7, "double")
    add("basic_byte_x1", 1, "byte")
    return c


def main():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cs = cases()
    names = [n for n, _, _ in cs]
    assert len(names) == len(set(names)), "duplicate case names"
    with open(OUT, "w") as f:
        f.write("# name | count | recipe   (generated by tools/make_cases.py)\n")
        for n, k, r in cs:
            f.write(f"{n} | {k} | {r}\n")
    print(f"wrote {len(cs)} cases to {OUT}")


if __name__ == "__main__":
    main()
