/* fd_txn_parse_core.h -- fd_txn_parse restated once, compiled twice: into
   the host library (host/fd_ed25519_hip_tile.c, gcc) and into the device
   staging kernel (fd_ed25519_txn.hip, hipcc), so both accept exactly the
   same payloads.  The includer defines FD_TXN_FN (the function qualifiers)
   and provides fd_ed25519_hip_txn_t (include/fd_ed25519_hip_tile.h).

   Reference: src/ballet/txn/fd_txn_parse.c:6-244 (fd_txn_parse_core with
   allow_zero_signatures=0 and no trailing bytes, i.e. fd_txn_parse), and
   the compact-u16 rules of src/ballet/txn/fd_compact_u16.h.  Each rule
   below is the reference's CHECK at the cited line; a payload is accepted
   iff every rule holds.  Offsets are read only after the bytes are known
   to be present.

   Besides the summary fields (fd_ed25519_hip_txn_t), the parser can write
   the reference's fd_txn_t itself, byte for byte (src/ballet/txn/fd_txn.h:
   the 20-byte header, instr[instr_cnt] of 10 bytes, then the address
   table lookups of 8 bytes, fd_txn_get_address_tables; little-endian,
   padding bytes zero as fd_txn_parse writes them), into `full`: the
   trailer the verify tile publishes behind the payload
   (src/app/fdctl/run/tiles/fd_verify.c:102-133).  Entries past full_cap
   bytes are not written (the header always is, so a reader of a short
   buffer sees the footprint). */
#ifndef FD_TXN_PARSE_CORE_H
#define FD_TXN_PARSE_CORE_H

#ifndef FD_TXN_FN
#define FD_TXN_FN static inline
#endif

#define FD_TXN_CORE_MTU       1232UL
#define FD_TXN_CORE_SIG_MAX    127UL
#define FD_TXN_CORE_ACCT_MAX   128UL
#define FD_TXN_CORE_INSTR_MAX   64UL
#define FD_TXN_CORE_LUT_MAX    127UL
#define FD_TXN_CORE_MAX_SZ     852UL   /* FD_TXN_MAX_SZ, fd_txn.h */

/* fd_txn_footprint (src/ballet/txn/fd_txn.h): header, instructions, LUTs */
#define FD_TXN_CORE_FOOTPRINT( instr_cnt, lut_cnt ) (20UL + 10UL*(unsigned long)(instr_cnt) + 8UL*(unsigned long)(lut_cnt))

FD_TXN_FN void
fd_txn_core_st16( unsigned char * d, unsigned long v ) {
  d[0] = (unsigned char)v;
  d[1] = (unsigned char)(v >> 8);
}

/* compact-u16: 1-3 bytes, 7 bits per byte little-endian, minimal encoding
   required; returns the encoded size (0: malformed / truncated) */
FD_TXN_FN unsigned long
fd_txn_core_cu16( unsigned char const * b, unsigned long avail, unsigned * val ) {
  if( avail>=1UL && !(b[0] & 0x80U) ) { *val = b[0]; return 1UL; }
  if( avail>=2UL && !(b[1] & 0x80U) ) {
    if( !b[1] ) return 0UL;                                      /* non-minimal */
    *val = (b[0] & 0x7FU) | ((unsigned)b[1] << 7);
    return 2UL;
  }
  if( avail>=3UL && !(b[2] & 0xFCU) ) {
    if( !b[2] ) return 0UL;                                      /* non-minimal */
    *val = (b[0] & 0x7FU) | ((unsigned)(b[1] & 0x7FU) << 7) | ((unsigned)b[2] << 14);
    return 3UL;
  }
  return 0UL;
}

/* Returns fd_txn_t's footprint (0: rejected).  out (optional): the summary
   fields; full (optional, full_cap >= 20): fd_txn_t bytes, the entries
   that fit in full_cap bytes and always the header. */
FD_TXN_FN unsigned long
fd_txn_core_parse( unsigned char const * p, unsigned long sz, fd_ed25519_hip_txn_t * out, unsigned char * full,
                   unsigned long full_cap ) {
  unsigned long i = 0UL, n;
  unsigned v;
#define HAVE( k ) ( (unsigned long)(k) <= sz - i )
#define CU16( dst ) do { n = fd_txn_core_cu16( p + i, sz - i, &v ); if( !n ) return 0; (dst) = v; i += n; } while(0)
  if( sz>FD_TXN_CORE_MTU ) return 0;                                                     /* :85 */
  if( !HAVE( 1 ) ) return 0;
  unsigned sig_cnt = p[ i++ ];
  if( sig_cnt<1U || sig_cnt>FD_TXN_CORE_SIG_MAX ) return 0;                              /* :94 */
  if( !HAVE( 64UL*sig_cnt ) ) return 0;
  unsigned long sig_off = i;  i += 64UL*sig_cnt;
  unsigned long msg_off = i;
  if( !HAVE( 1 ) ) return 0;
  unsigned b0 = p[ i++ ];
  unsigned char ver;
  if( b0 & 0x80U ) {                                                                     /* :102-107 */
    ver = (unsigned char)(b0 & 0x7FU);
    if( ver!=0U ) return 0;
    if( !HAVE( 1 ) ) return 0;
    if( p[ i ]!=sig_cnt ) return 0;
    i++;
  } else {
    ver = 0xFF;
    if( b0!=sig_cnt ) return 0;                                                          /* :110 */
  }
  if( !HAVE( 1 ) ) return 0;
  unsigned ro_signed = p[ i++ ];
  if( !(ro_signed<sig_cnt) ) return 0;                                                   /* :114 */
  if( !HAVE( 1 ) ) return 0;
  unsigned ro_unsigned = p[ i++ ];
  unsigned acct_cnt;  CU16( acct_cnt );
  if( !(sig_cnt<=acct_cnt && acct_cnt<=FD_TXN_CORE_ACCT_MAX) ) return 0;                 /* :120 */
  if( sig_cnt + ro_unsigned > acct_cnt ) return 0;                                       /* :121 */
  if( !HAVE( 32UL*acct_cnt ) ) return 0;
  unsigned long acct_off = i;  i += 32UL*acct_cnt;
  if( !HAVE( 32 ) ) return 0;
  unsigned long bh_off = i;  i += 32UL;
  unsigned instr_cnt;  CU16( instr_cnt );
  if( instr_cnt>FD_TXN_CORE_INSTR_MAX ) return 0;                                        /* :132 */
  if( !HAVE( 3UL*instr_cnt ) ) return 0;                                                 /* :133 */
  if( !(acct_cnt > (instr_cnt ? 1U : 0U)) ) return 0;                                    /* :136 */
  unsigned max_acct = 0U;
  for( unsigned j=0U; j<instr_cnt; j++ ) {
    if( !HAVE( 3 ) ) return 0;
    unsigned prog = p[ i++ ];
    unsigned ia; CU16( ia );
    if( !HAVE( ia ) ) return 0;
    unsigned long ia_off = i;
    for( unsigned k=0U; k<ia; k++ ) if( p[ i+k ]>max_acct ) max_acct = p[ i+k ];
    i += ia;
    unsigned dsz; CU16( dsz );
    if( !HAVE( dsz ) ) return 0;
    unsigned long d_off = i;
    i += dsz;
    if( !(0U<prog && prog<acct_cnt) ) return 0;                                          /* :175 */
    if( full && 20UL + 10UL*(j+1UL)<=full_cap ) {                                        /* :177-186 */
      unsigned char * e = full + 20UL + 10UL*j;
      e[0] = (unsigned char)prog; e[1] = 0;
      fd_txn_core_st16( e+2, ia ); fd_txn_core_st16( e+4, dsz );
      fd_txn_core_st16( e+6, ia_off ); fd_txn_core_st16( e+8, d_off );
    }
  }
  unsigned lut_cnt = 0U;
  unsigned long adtl = 0UL, adtl_w = 0UL;
  if( ver==0U ) {
    CU16( lut_cnt );
    if( lut_cnt>FD_TXN_CORE_LUT_MAX ) return 0;                                          /* :199 */
    if( !HAVE( 34UL*lut_cnt ) ) return 0;
    for( unsigned j=0U; j<lut_cnt; j++ ) {
      if( !HAVE( 32 ) ) return 0;
      unsigned long a_off = i;
      i += 32UL;
      unsigned w, r;
      CU16( w );  if( !HAVE( w ) ) return 0;  unsigned long w_off = i;  i += w;
      CU16( r );  if( !HAVE( r ) ) return 0;  unsigned long r_off = i;  i += r;
      if( w > FD_TXN_CORE_ACCT_MAX - acct_cnt ) return 0;                                /* :212 */
      if( r > FD_TXN_CORE_ACCT_MAX - acct_cnt ) return 0;
      if( w + r < 1U ) return 0;
      if( full && FD_TXN_CORE_FOOTPRINT( instr_cnt, j+1U )<=full_cap ) {                 /* :216-222 */
        unsigned char * e = full + FD_TXN_CORE_FOOTPRINT( instr_cnt, j );
        fd_txn_core_st16( e, a_off ); e[2] = (unsigned char)w; e[3] = (unsigned char)r;
        fd_txn_core_st16( e+4, w_off ); fd_txn_core_st16( e+6, r_off );
      }
      adtl_w += w;
      adtl   += (unsigned long)w + r;
    }
  }
  if( i!=sz ) return 0;                                                                  /* :229 */
  if( acct_cnt + adtl > FD_TXN_CORE_ACCT_MAX ) return 0;                                 /* :231 */
  if( !(max_acct < acct_cnt + adtl) ) return 0;                                          /* :234 */
#undef HAVE
#undef CU16
  if( out ) {
    out->transaction_version          = ver;
    out->signature_cnt                = (unsigned char)sig_cnt;
    out->signature_off                = (unsigned short)sig_off;
    out->message_off                  = (unsigned short)msg_off;
    out->readonly_signed_cnt          = (unsigned char)ro_signed;
    out->readonly_unsigned_cnt        = (unsigned char)ro_unsigned;
    out->acct_addr_cnt                = (unsigned short)acct_cnt;
    out->acct_addr_off                = (unsigned short)acct_off;
    out->recent_blockhash_off         = (unsigned short)bh_off;
    out->instr_cnt                    = (unsigned short)instr_cnt;
    out->addr_table_lookup_cnt        = (unsigned char)lut_cnt;
    out->addr_table_adtl_writable_cnt = (unsigned char)adtl_w;
    out->addr_table_adtl_cnt          = (unsigned char)adtl;
  }
  unsigned long foot = FD_TXN_CORE_FOOTPRINT( instr_cnt, lut_cnt );
  /* the header always (it tells a reader of a short buffer the footprint:
     instr_cnt at 18, addr_table_lookup_cnt at 14) */
  if( full && full_cap>=20UL ) {                                                         /* :145-157, :238-243 */
    full[0] = ver;                              full[1] = (unsigned char)sig_cnt;
    fd_txn_core_st16( full+2,  sig_off );       fd_txn_core_st16( full+4,  msg_off );
    full[6] = (unsigned char)ro_signed;         full[7] = (unsigned char)ro_unsigned;
    fd_txn_core_st16( full+8,  acct_cnt );      fd_txn_core_st16( full+10, acct_off );
    fd_txn_core_st16( full+12, bh_off );
    full[14] = (unsigned char)lut_cnt;          full[15] = (unsigned char)adtl_w;
    full[16] = (unsigned char)adtl;             full[17] = 0;
    fd_txn_core_st16( full+18, instr_cnt );
  }
  return foot;
}

#endif
