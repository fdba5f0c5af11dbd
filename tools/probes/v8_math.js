// V8's own Math.cos / Math.sin / Math.pow (the JS engine's built-ins - no
// reference code) at the arguments the path tracer feeds them: the cosine-PDF
// angle phi = 2 * Math.PI * xi and Schlick's Math.pow(1 - cos, 5)
// (src/geometry/vec3.ts:325-337, src/materials/dielectric.ts:98), with
// xi = u / 2^32 for a deterministic u32 sequence. Writes little-endian records
// {u32 u, f64 cos(phi), f64 sin(phi), f64 pow(xi, 5)} to argv[3].
'use strict';
const fs = require('fs');
const n = parseInt(process.argv[2], 10);
const buf = Buffer.alloc(n * 28);
let s = 0x5eed >>> 0;
for (let k = 0; k < n; ++k) {
  s = (Math.imul(s, 1664525) + 1013904223) >>> 0;
  const xi = s * (1 / 4294967296);
  const phi = 2 * Math.PI * xi;
  const o = k * 28;
  buf.writeUInt32LE(s, o);
  buf.writeDoubleLE(Math.cos(phi), o + 4);
  buf.writeDoubleLE(Math.sin(phi), o + 12);
  buf.writeDoubleLE(Math.pow(xi, 5), o + 20);
}
fs.writeFileSync(process.argv[3], buf);
