// Node-side harness for the N-API addon (this repo's own test code, not the
// reference): the calls the reference's TypeScript host would make through
// INTEGRATION.md's binding. usage:
//   node addon_render.js <addon.node> info            -> JSON camera info (no GPU)
//   node addon_render.js <addon.node> render <out.bin> -> JSON stats, RGB bytes to out.bin (+ .png, .dev.png)
//   node addon_render.js <addon.node> errors           -> JSON list of thrown messages
'use strict';
const fs = require('fs');
const addon = require(process.argv[2]);
const mode = process.argv[3];

const sceneJson = addon.generateSceneData('cornell', null);
const scene = JSON.parse(sceneJson);
const opts = { width: 40, samples: 8, depth: 8, aTolerance: 0 };

if (mode === 'info') {
  const cam = addon.createCamera(sceneJson, JSON.stringify(opts));
  const info = addon.cameraInfo(cam);
  console.log(JSON.stringify({ version: addon.version(), objects: scene.objects.length, info }));
} else if (mode === 'render') {
  const cam = addon.createCamera(sceneJson, JSON.stringify(opts));
  const info = addon.cameraInfo(cam);
  // generateImageBuffer's parallel path hands each worker a region of one shared buffer
  const shared = new SharedArrayBuffer(info.imageWidth * info.imageHeight * 3);
  const pixels = new Uint8ClampedArray(shared);
  const half = Math.ceil(info.imageHeight / 2);
  const s1 = addon.renderRegion(cam, pixels, { x: 0, y: 0, width: info.imageWidth, height: half });
  const s2 = addon.renderRegion(cam, pixels, { x: 0, y: half, width: info.imageWidth, height: info.imageHeight - half });
  fs.writeFileSync(process.argv[4], Buffer.from(shared));
  fs.writeFileSync(process.argv[4] + '.png', addon.encodePng(pixels, info.imageWidth, info.imageHeight));
  // generateImageBuffer's core on the device: 3 worker bands, PNG encoded on the GPU
  const dev = addon.renderPng(cam, 3);
  fs.writeFileSync(process.argv[4] + '.dev.png', dev.png);
  // the workers' fan-out as one call over GPUs of this process: device 0 listed 3 times
  // (the split rehearsed on one GPU), then every visible GPU given as a count
  const multi = new Uint8ClampedArray(info.imageWidth * info.imageHeight * 3);
  const sm = addon.renderRegionMulti(cam, multi, { x: 0, y: 0, width: info.imageWidth, height: info.imageHeight },
                                     [0, 0, 0]);
  fs.writeFileSync(process.argv[4] + '.multi', Buffer.from(multi.buffer));
  const devm = addon.renderPng(cam, 1, Number(process.argv[5] || 1));
  fs.writeFileSync(process.argv[4] + '.multi.png', devm.png);
  console.log(JSON.stringify({ width: info.imageWidth, height: info.imageHeight, stats: [s1, s2], devStats: dev.stats,
                               multiStats: sm, multiPngStats: devm.stats }));
} else if (mode === 'png') {
  // host-only: encodePng of a synthetic frame (no GPU)
  const w = 5, h = 3;
  const px = new Uint8ClampedArray(w * h * 3);
  for (let k = 0; k < px.length; ++k) px[k] = (k * 7) % 251;
  fs.writeFileSync(process.argv[4], addon.encodePng(px, w, h));
  console.log(JSON.stringify({ width: w, height: h }));
} else if (mode === 'errors') {
  const msgs = [];
  const bad = JSON.parse(sceneJson);
  bad.objects[0].material = 'nope';
  try { addon.createCamera(JSON.stringify(bad)); } catch (e) { msgs.push(e.message); }
  bad.objects[0].material = scene.objects[0].material;
  bad.objects[0].type = 'torus';
  try { addon.createCamera(JSON.stringify(bad)); } catch (e) { msgs.push(e.message); }
  try { addon.renderRegion({}, new Uint8ClampedArray(3), { x: 0, y: 0, width: 1, height: 1 }); } catch (e) { msgs.push(e.message); }
  console.log(JSON.stringify(msgs));
} else {
  throw new Error('unknown mode ' + mode);
}
