// Cross-checks tests/golden/golden.json with Node's crypto SHA-1 (an SHA-1
// independent of Python hashlib and of oracle/bf_oracle.c):
//   node tests/golden/crosscheck_node.js
// Restates lib/bloomfilter_driver/ruby.rb:41-55 with BigInt arithmetic.
'use strict';
const crypto = require('crypto');
const fs = require('fs');
const path = require('path');

const g = JSON.parse(fs.readFileSync(path.join(__dirname, 'golden.json'), 'utf8'));

function indexes(buf, m, k) {
  const hex = crypto.createHash('sha1').update(buf).digest('hex');
  const h = [0, 1, 2, 3].map((j) => BigInt('0x' + hex.slice(8 * j, 8 * j + 8)));
  const out = [];
  for (let i = 0; i < k; ++i) {
    const a = h[i % 2];
    const b = h[2 + Math.floor(((i + (i % 2)) % 4) / 2)];
    out.push(((a + BigInt(i) * b) % BigInt(m)).toString());
  }
  return out;
}

// lib/bloomfilter_driver/ruby_test.rb:55-61: hexdigest("#{i}-#{data}").to_i(16) % bits
function engineIndexes(engine, buf, m, k) {
  const out = [];
  for (let i = 0; i < k; ++i) {
    const hex = crypto.createHash(engine).update(Buffer.concat([Buffer.from(i + '-'), buf])).digest('hex');
    out.push((BigInt('0x' + hex) % BigInt(m)).toString());
  }
  return out;
}

let bad = 0;
for (const [msg, want] of Object.entries(g.rfc1321_md5)) {
  if (crypto.createHash('md5').update(Buffer.from(msg, 'latin1')).digest('hex') !== want) bad++;
}
for (const v of g.engine_indexes) {
  const got = engineIndexes(v.engine, Buffer.from(v.key_hex, 'hex'), v.m, v.k);
  if (got.join(',') !== v.idx.map(String).join(',')) { bad++; console.log('engine mismatch', v.engine, v.key_hex, v.m); }
}
for (const [msg, want] of Object.entries(g.fips_sha1)) {
  if (crypto.createHash('sha1').update(Buffer.from(msg, 'latin1')).digest('hex') !== want) bad++;
}
for (const v of g.indexes) {
  const got = indexes(Buffer.from(v.key_hex, 'hex'), v.m, v.k);
  if (got.join(',') !== v.idx.map(String).join(',')) { bad++; console.log('mismatch', v.key_hex, v.m, v.k); }
}
for (const s of g.strings) {
  const bytes = new Map();
  let maxByte = -1;
  for (const key of s.insert) {
    for (const o of indexes(Buffer.from(key, 'utf8'), s.m, s.k)) {
      const off = BigInt(o);
      const byte = Number(off >> 3n);
      bytes.set(byte, (bytes.get(byte) || 0) | (0x80 >> Number(off & 7n)));
      if (byte > maxByte) maxByte = byte;
    }
  }
  const buf = Buffer.alloc(maxByte + 1);
  for (const [b, v] of bytes) buf[b] = v;
  const sha = crypto.createHash('sha1').update(buf).digest('hex');
  if (sha !== s.redis_sha1 || buf.length !== s.redis_len) { bad++; console.log('string mismatch', s.name); }
}
console.log(bad === 0 ? 'node crosscheck ok (' + g.indexes.length + ' index vectors, ' + g.engine_indexes.length +
                        ' engine vectors, ' + g.strings.length + ' strings)'
                      : 'node crosscheck FAILED: ' + bad);
process.exit(bad === 0 ? 0 : 1);
