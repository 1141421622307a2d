{-# LANGUAGE ForeignFunctionInterface #-}
-- |
-- Module      : RenderAMD
-- Description : runRender (src/Lib.hs:1491) on an AMD MI355X through the C ABI of include/rt.h
--
-- The module a maintainer of the reference would add as src/RenderAMD.hs to render on the GPU:
-- it flattens the reference's own values ('Scene' = (world, lights, background), src/Lib.hs:84;
-- 'Camera', src/Lib.hs:1230-1251; '[RandGen]', src/Random.hs:11-12) into the plain records of
-- include/rt.h and calls librtamd.so.
--
-- UNTESTED AS HASKELL: no GHC exists in the build image or on the GPU box (SURVEY.md §0.2), so this
-- file has never been compiled. Its call sequence — post-order flattening of the Hittable tree into
-- an rt_scene_desc, rt_create on GPU 0 (or, opt-in for tier B, rt_create_multi over n GPUs),
-- rt_upload_scene, rt_render (tier A, one SplitMix generator per column; tier B one Philox stream per
-- pixel and sample, tile-sharded over the GPUs and gathered with RCCL inside librtamd on a multi-GPU
-- ctx), rows split top first, rt_destroy — is mirrored in C by
-- tests/c/ffi_sequence.c, which tests/test_ffi_sequence.py compiles and runs (the rendering half on the
-- GPU, checked against the CPU oracle on the same flattened records).
--
-- What the reference package needs for it (integration/reference.patch, a `patch -p1` against the
-- reference's root; then copy this file to src/RenderAMD.hs):
--   * src/Lib.hs export list (lines 4-51): @Camera(..)@ instead of the abstract @Camera@ (line 39),
--     and @Rectangle(..)@ and @RGB(..)@ (not exported), so that cameras, rectangles and output
--     pixels can be taken apart / built here;
--   * package.yaml library dependencies (lines 25-35): add @splitmix@ — this module imports
--     "System.Random.SplitMix" ('unseedSMGen'), and splitmix is only pinned as an extra-dep
--     (stack.yaml:42-44), not a dependency of the library; random-1.2.0's
--     "System.Random.Internal" ('StdGen' / 'unStdGen'), JuicyPixels ("Codec.Picture"), mtl and vector
--     already are dependencies (package.yaml:27-35);
--   * package.yaml library: @extra-libraries: rtamd@, @extra-lib-dirs@ at ray-tracing_amd/build
--     (librtamd.so pulls the ROCm runtime, libamdhip64) and @include-dirs@ at include/, through a
--     link `rtamd` to this repository's checkout.
module RenderAMD
  ( -- * Drop-ins for runRender
    runRenderAMD
  , runRenderAMDPhilox
  , runRenderAMDPhiloxOn
    -- * The flattened scene (include/rt.h records)
  , FlatScene (..)
  , RtNode (..)
  , RtMat (..)
  , RtTex (..)
  , RtPerlin (..)
  , RtImage (..)
  , flattenScene
  , withSceneDesc
  , columnGens
  , RtError (..)
  ) where

import qualified Codec.Picture              as JP
import           Control.Exception          (Exception, bracket, throwIO)
import           Control.Monad              (when, zipWithM_)
import           Control.Monad.State.Strict (State, get, put, runState)
import qualified Data.Vector                as VV
import qualified Data.Vector.Storable       as SV
import qualified Data.Vector.Storable.Mutable as SVM
import qualified Data.Vector.Unboxed        as VU
import           Foreign
import           Foreign.C.String           (CString, peekCString)
import           Foreign.C.Types            (CInt (..))
import           Lib                        hiding (length, rotate)
import           Random                     (RandGen (..))
import           System.Random.Internal     (StdGen (..))
import           System.Random.SplitMix     (unseedSMGen)

-- ---------------------------------------------------------------- the C ABI (include/rt.h)
data RtCtx
data SceneDesc     -- rt_scene_desc, 112 bytes
data CameraRec     -- rt_camera, 192 bytes
data RenderParams  -- rt_render_params, 48 bytes

foreign import ccall unsafe "rt.h rt_device_count"
  c_rt_device_count :: Ptr CInt -> IO CInt
-- one ctx on one GPU (the default: runRenderAMD, runRenderAMDPhilox)
foreign import ccall unsafe "rt.h rt_create"
  c_rt_create :: CInt -> Ptr (Ptr RtCtx) -> IO CInt
-- one ctx over n GPUs (NULL device list = 0..n-1): tier-B frames shard over them, RCCL gathers
-- (runRenderAMDPhiloxOn, opt-in)
foreign import ccall unsafe "rt.h rt_create_multi"
  c_rt_create_multi :: CInt -> Ptr CInt -> Ptr (Ptr RtCtx) -> IO CInt
foreign import ccall unsafe "rt.h rt_destroy"
  c_rt_destroy :: Ptr RtCtx -> IO ()
foreign import ccall safe "rt.h rt_upload_scene"
  c_rt_upload_scene :: Ptr RtCtx -> Ptr SceneDesc -> IO CInt
-- rt_render blocks for the whole frame: a safe call, so the RTS keeps running other threads.
foreign import ccall safe "rt.h rt_render"
  c_rt_render :: Ptr RtCtx -> Ptr CameraRec -> Ptr RenderParams -> Ptr Word64 -> Ptr Word8
              -> Ptr Double -> Ptr Word64 -> IO CInt
foreign import ccall unsafe "rt.h rt_last_error"
  c_rt_last_error :: IO CString

-- | A negative RT_E* code and rt_last_error()'s message.
data RtError = RtError String Int deriving (Show)
instance Exception RtError

check :: String -> IO CInt -> IO ()
check what act = do
  rc <- act
  when (rc < 0) $ do
    msg <- c_rt_last_error >>= peekCString
    throwIO (RtError (what ++ ": " ++ msg) (fromIntegral rc))

rtRngExact, rtRngPhilox :: Int32
rtRngExact = 0   -- RT_RNG_EXACT: the reference's per-column SplitMix streams (runRender's layout)
rtRngPhilox = 1  -- RT_RNG_PHILOX: per (pixel, sample) Philox streams (the fast path)

-- ---------------------------------------------------------------- flattened records
-- | rt_node: up to 6 doubles, type, a, b, c (the c field is htblSize, src/Lib.hs:662-671).
data RtNode = RtNode ![Double] !Int32 !Int32 !Int32 !Int32
-- | rt_material: type, texture id, param (fuzz / refractive index).
data RtMat = RtMat !Int32 !Int32 !Double
-- | rt_texture: type, a, b, c, up to 4 doubles.
data RtTex = RtTex !Int32 !Int32 !Int32 !Int32 ![Double]
-- | rt_perlin: ranvec (256 x 3), perm_x, perm_y, perm_z (256 each).
data RtPerlin = RtPerlin ![Double] ![Int32] ![Int32] ![Int32]
-- | rt_image: byte offset into the pool, width, height.
data RtImage = RtImage !Int64 !Int32 !Int32

-- | A flattened 'Scene': children precede their parents (rt_upload_scene checks it, which also
-- makes the graph acyclic). Haskell sharing (the Cornell light in both trees, BVHNode h h, a
-- medium's boundary also in the world) becomes one copy per occurrence.
data FlatScene = FlatScene
  { fsNodes      :: [RtNode]
  , fsMats       :: [RtMat]
  , fsTexs       :: [RtTex]
  , fsPerlins    :: [RtPerlin]
  , fsImages     :: [RtImage]
  , fsPool       :: SV.Vector Word8  -- RGB8 rasters, concatenated in image order
  , fsWorld      :: Int32
  , fsLights     :: Int32            -- -1 = Unhittable (rt_scene_desc.lights_root)
  , fsBackground :: [Double]
  }

data Acc = Acc
  { aNodes :: [RtNode], aN :: !Int32
  , aMats :: [RtMat], aM :: !Int32
  , aTexs :: [RtTex], aT :: !Int32
  , aPerlins :: [RtPerlin], aP :: !Int32
  , aImages :: [RtImage], aI :: !Int32
  , aPool :: [SV.Vector Word8], aPoolBytes :: !Int64
  }

emptyAcc :: Acc
emptyAcc = Acc [] 0 [] 0 [] 0 [] 0 [] 0 [] 0

emitNode :: RtNode -> State Acc Int32
emitNode x = do
  a <- get
  put a {aNodes = x : aNodes a, aN = aN a + 1}
  return (aN a)

emitMat :: RtMat -> State Acc Int32
emitMat x = do
  a <- get
  put a {aMats = x : aMats a, aM = aM a + 1}
  return (aM a)

emitTex :: RtTex -> State Acc Int32
emitTex x = do
  a <- get
  put a {aTexs = x : aTexs a, aT = aT a + 1}
  return (aT a)

emitPerlin :: RtPerlin -> State Acc Int32
emitPerlin x = do
  a <- get
  put a {aPerlins = x : aPerlins a, aP = aP a + 1}
  return (aP a)

-- | The raster of an ImageTexture, row 0 = top, RGB8 (JuicyPixels' imageData layout, which is
-- what pixelAt indexes, src/Lib.hs:386-389).
emitImage :: JP.Image JP.PixelRGB8 -> State Acc Int32
emitImage im = do
  a <- get
  let bytes = JP.imageData im
      recd = RtImage (aPoolBytes a) (fromIntegral (JP.imageWidth im)) (fromIntegral (JP.imageHeight im))
  put a { aImages = recd : aImages a, aI = aI a + 1
        , aPool = bytes : aPool a, aPoolBytes = aPoolBytes a + fromIntegral (SV.length bytes) }
  return (aI a)

v3 :: Vec3 -> [Double]
v3 v = [vecX v, vecY v, vecZ v]

-- | htblSize (src/Lib.hs:662-671), restated: Lib does not export it.
hSize :: Hittable -> Int32
hSize h = case h of
  Unhittable          -> 0
  BVHNode _ _ _ n     -> fromIntegral n
  Translate _ c       -> hSize c
  Rotate _ _ _ _ c    -> hSize c
  _                   -> 1

axisId :: Axis -> Int32
axisId XAxis = 0
axisId YAxis = 1
axisId ZAxis = 2

-- | Texture (src/Lib.hs:394-419) -> rt_texture (+ Perlin table / image raster). Checker children
-- are emitted first (rt_upload_scene: they must precede the checker).
flatTex :: Texture -> State Acc Int32
flatTex t = case t of
  ConstantColor (Albedo c) -> emitTex (RtTex 0 0 0 0 (v3 c))
  CheckerTexture oddT evenT -> do
    io <- flatTex oddT
    ie <- flatTex evenT
    emitTex (RtTex 1 io ie 0 [])
  Perlin ranvec px py pz sc -> do
    ip <- emitPerlin (RtPerlin (concatMap v3 (VV.toList ranvec)) (perm px) (perm py) (perm pz))
    emitTex (RtTex 2 ip 0 0 [sc])
  ImageTexture Nothing nx ny -> emitTex (RtTex 3 (-1) (fromIntegral nx) (fromIntegral ny) [])
  ImageTexture (Just (Image im)) nx ny -> do
    ii <- emitImage im
    emitTex (RtTex 3 ii (fromIntegral nx) (fromIntegral ny) [])
  where
    perm = map fromIntegral . VU.toList

-- | Material (src/Lib.hs:339-345) -> rt_material.
flatMat :: Material -> State Acc Int32
flatMat m = case m of
  Lambertian t                  -> flatTex t >>= \it -> emitMat (RtMat 0 it 0)
  Metal t (Fuzz f)              -> flatTex t >>= \it -> emitMat (RtMat 1 it f)
  Dielectric (RefractiveIdx ri) -> emitMat (RtMat 2 (-1) ri)
  DiffuseLight t                -> flatTex t >>= \it -> emitMat (RtMat 3 it 0)
  Isotropic t                   -> flatTex t >>= \it -> emitMat (RtMat 4 it 0)

-- | Rectangle (src/Lib.hs:607-647) -> (rt_node type, fields in the constructor's order, material).
rectRec :: Rectangle -> (Int32, [Double], Material)
rectRec r = case r of
  XYRect x0 x1 y0 y1 k mat -> (3, [x0, x1, y0, y1, k], mat)
  XZRect x0 x1 z0 z1 k mat -> (4, [x0, x1, z0, z1, k], mat)
  YZRect y0 y1 z0 z1 k mat -> (5, [y0, y1, z0, z1, k], mat)

-- | Hittable (src/Lib.hs:521-585) -> rt_node records, post-order (children first).
flatHit :: Hittable -> State Acc Int32
flatHit h = case h of
  BVHNode l r (Box bmin bmax) n -> do
    il <- flatHit l
    ir <- flatHit r
    emitNode (RtNode (v3 bmin ++ v3 bmax) 0 il ir (fromIntegral n))
  Sphere c rad mat -> do
    im <- flatMat mat
    emitNode (RtNode (v3 c ++ [rad]) 1 im 0 1)
  MovingSphere c0 c1 t0 t1 dur rad mat -> do
    im <- flatMat mat
    i <- emitNode (RtNode (v3 c0 ++ v3 c1) 2 im 0 1)
    _ <- emitNode (RtNode [t0, t1, dur, rad] 11 0 0 0)  -- RT_NODE_EXT, right after its sphere
    return i
  Rect r -> do
    let (ty, fs, mat) = rectRec r
    im <- flatMat mat
    emitNode (RtNode fs ty im 0 1)
  -- The device rebuilds the six faces from min/max in cuboid's order (src/Lib.hs:599-604), so only
  -- the shared material is kept: every Cuboid the reference builds comes from `cuboid`.
  Cuboid bmin bmax (face : _) -> do
    let (_, _, mat) = rectRec face
    im <- flatMat mat
    emitNode (RtNode (v3 bmin ++ v3 bmax) 6 im 0 1)
  Cuboid _ _ [] -> error "RenderAMD: a Cuboid without faces cannot come from `cuboid`"
  Translate off c -> do
    ic <- flatHit c
    emitNode (RtNode (v3 off) 7 ic 0 (hSize c))
  Rotate ax s co _ c -> do
    ic <- flatHit c
    emitNode (RtNode [s, co] 8 ic (axisId ax) (hSize c))
  ConstantMedium negInvDensity mat boundary -> do
    ib <- flatHit boundary
    im <- flatMat mat
    emitNode (RtNode [negInvDensity] 9 ib im 1)
  Unhittable -> emitNode (RtNode [] 10 0 0 0)

-- | Flatten a 'Scene' (src/Lib.hs:84). An Unhittable lights tree becomes lights_root = -1 (what
-- htblRandom / htblPdfValue do with it, src/Lib.hs:702,724, is what the device does for -1).
flattenScene :: Scene -> FlatScene
flattenScene (world, lights, Albedo bg) =
  let go = do
        w <- flatHit world
        l <- case lights of
          Unhittable -> return (-1)
          _          -> flatHit lights
        return (w, l)
      ((w, l), acc) = runState go emptyAcc
   in FlatScene
        { fsNodes = reverse (aNodes acc), fsMats = reverse (aMats acc), fsTexs = reverse (aTexs acc)
        , fsPerlins = reverse (aPerlins acc), fsImages = reverse (aImages acc)
        , fsPool = SV.concat (reverse (aPool acc)), fsWorld = w, fsLights = l, fsBackground = v3 bg }

-- ---------------------------------------------------------------- Storable records (rt.h layout)
instance Storable RtNode where
  sizeOf _ = 64
  alignment _ = 8
  peek p = do
    fs <- peekArray 6 (castPtr p :: Ptr Double)
    RtNode fs <$> peekByteOff p 48 <*> peekByteOff p 52 <*> peekByteOff p 56 <*> peekByteOff p 60
  poke p (RtNode fs ty a b c) = do
    pokeArray (castPtr p :: Ptr Double) (take 6 (fs ++ repeat 0))
    pokeByteOff p 48 ty
    pokeByteOff p 52 a
    pokeByteOff p 56 b
    pokeByteOff p 60 c

instance Storable RtMat where
  sizeOf _ = 16
  alignment _ = 8
  peek p = RtMat <$> peekByteOff p 0 <*> peekByteOff p 4 <*> peekByteOff p 8
  poke p (RtMat ty tex param) = pokeByteOff p 0 ty >> pokeByteOff p 4 tex >> pokeByteOff p 8 param

instance Storable RtTex where
  sizeOf _ = 48
  alignment _ = 8
  peek p = do
    fs <- peekArray 4 (castPtr p `plusPtr` 16 :: Ptr Double)
    RtTex <$> peekByteOff p 0 <*> peekByteOff p 4 <*> peekByteOff p 8 <*> peekByteOff p 12 <*> pure fs
  poke p (RtTex ty a b c fs) = do
    pokeByteOff p 0 ty
    pokeByteOff p 4 a
    pokeByteOff p 8 b
    pokeByteOff p 12 c
    pokeArray (castPtr p `plusPtr` 16 :: Ptr Double) (take 4 (fs ++ repeat 0))

instance Storable RtPerlin where
  sizeOf _ = 9216
  alignment _ = 8
  peek p = RtPerlin <$> peekArray 768 (castPtr p) <*> peekArray 256 (castPtr p `plusPtr` 6144)
                    <*> peekArray 256 (castPtr p `plusPtr` 7168) <*> peekArray 256 (castPtr p `plusPtr` 8192)
  poke p (RtPerlin ranvec px py pz) = do
    pokeArray (castPtr p :: Ptr Double) ranvec
    pokeArray (castPtr p `plusPtr` 6144 :: Ptr Int32) px
    pokeArray (castPtr p `plusPtr` 7168 :: Ptr Int32) py
    pokeArray (castPtr p `plusPtr` 8192 :: Ptr Int32) pz

instance Storable RtImage where
  sizeOf _ = 16
  alignment _ = 8
  peek p = RtImage <$> peekByteOff p 0 <*> peekByteOff p 8 <*> peekByteOff p 12
  poke p (RtImage off w h) = pokeByteOff p 0 off >> pokeByteOff p 8 w >> pokeByteOff p 12 h

-- | An rt_scene_desc (112 bytes) over the flattened arrays, valid inside the continuation
-- (rt_upload_scene copies everything it needs).
withSceneDesc :: FlatScene -> (Ptr SceneDesc -> IO a) -> IO a
withSceneDesc fs k =
  withArrayLen (fsNodes fs) $ \nn pn ->
  withArrayLen (fsMats fs) $ \nm pm ->
  withArrayLen (fsTexs fs) $ \nt pt ->
  withArrayLen (fsPerlins fs) $ \np pp ->
  withArrayLen (fsImages fs) $ \ni pim ->
  SV.unsafeWith (fsPool fs) $ \ppool ->
  allocaBytes 112 $ \d -> do
    fillBytes d 0 112
    pokeByteOff d 0 pn
    pokeByteOff d 8 (fromIntegral nn :: Int32)
    pokeByteOff d 12 (fsWorld fs)
    pokeByteOff d 16 (fsLights fs)
    pokeByteOff d 20 (fromIntegral nm :: Int32)
    pokeByteOff d 24 pm
    pokeByteOff d 32 pt
    pokeByteOff d 40 (fromIntegral nt :: Int32)
    pokeByteOff d 44 (fromIntegral np :: Int32)
    pokeByteOff d 48 pp
    pokeByteOff d 56 pim
    pokeByteOff d 64 (fromIntegral ni :: Int32)
    pokeByteOff d 72 ppool
    pokeByteOff d 80 (fromIntegral (SV.length (fsPool fs)) :: Int64)
    pokeArray (d `plusPtr` 88 :: Ptr Double) (take 3 (fsBackground fs ++ repeat 0))
    k (castPtr d)

-- | rt_camera (192 bytes): the Camera record's fields in order (src/Lib.hs:1230-1251).
withCamera :: Camera -> (Ptr CameraRec -> IO a) -> IO a
withCamera (Camera o llc horiz vert u v w lensRadius t0 t1) k =
  withArray (concatMap v3 [o, llc, horiz, vert, u, v, w] ++ [lensRadius, t0, t1]) (k . castPtr)

-- | rt_render_params (48 bytes); whole image (shard 0 of 1), default 8-pixel tiles.
withParams :: Int -> Int -> Int -> Int -> Int32 -> Word64 -> (Ptr RenderParams -> IO a) -> IO a
withParams w h ns maxDepth rng seed k =
  allocaBytes 48 $ \p -> do
    fillBytes p 0 48
    zipWithM_ (\off x -> pokeByteOff p off (fromIntegral x :: Int32)) [0, 4, 8, 12] [w, h, ns, maxDepth]
    pokeByteOff p 16 rng
    pokeByteOff p 20 (0 :: Word32)   -- flags
    pokeByteOff p 24 seed
    pokeByteOff p 32 (8 :: Int32)    -- tile
    pokeByteOff p 36 (0 :: Int32)    -- shard_rank
    pokeByteOff p 40 (1 :: Int32)    -- shard_count
    k (castPtr p)

-- | One (seed, gamma) pair per column: the SplitMix state inside each RandGen (random-1.2.0's
-- StdGen is a newtype over splitmix's SMGen; unseedSMGen returns its seed and gamma).
columnGens :: [RandGen] -> [Word64]
columnGens gens = concat [[s, g] | RandGen std <- gens, let (s, g) = unseedSMGen (unStdGen std)]

-- | Render on `gpus` GPUs (<= 1: device 0 alone, rt_create; n > 1: rt_create_multi over devices
-- 0..n-1, at most the visible ones — tier B's tile shards gathered by RCCL; tier A's per-column streams
-- do not shard, so a tier-A frame always renders on one GPU); the raw H x W x 3 bytes, top row first.
renderBytes :: Int -> Scene -> Camera -> (Int, Int) -> Int -> Int -> Int32 -> Word64 -> [Word64]
            -> IO (SV.Vector Word8)
renderBytes gpus scene cam (w, h) ns maxDepth rng seed gensW = do
  let flat = flattenScene scene
  bracket acquire c_rt_destroy $ \ctx -> do
    withSceneDesc flat $ \d -> check "rt_upload_scene" (c_rt_upload_scene ctx d)
    out <- SVM.new (w * h * 3)
    withCamera cam $ \pc ->
      withParams w h ns maxDepth rng seed $ \pp ->
      withArray (if null gensW then [0] else gensW) $ \pg ->
      SVM.unsafeWith out $ \po ->
        check "rt_render" (c_rt_render ctx pc pp (if rng == rtRngExact then pg else nullPtr) po nullPtr nullPtr)
    SV.unsafeFreeze out
  where
    acquire = alloca $ \pn -> alloca $ \pctx -> do
      check "rt_device_count" (c_rt_device_count pn)
      avail <- peek pn
      let n = minimum [fromIntegral (max 1 gpus), avail, 16]  -- (RT_MAX_DEVICES = 16)
      if n <= 1 || rng == rtRngExact
        then check "rt_create" (c_rt_create 0 pctx)
        else check "rt_create_multi" (c_rt_create_multi n nullPtr pctx)
      peek pctx

-- | Rows of pixels, top row first, each `cols` wide.
toRows :: Int -> Int -> Int -> SV.Vector Word8 -> [VV.Vector RGB]
toRows w h cols bytes =
  [ VV.generate cols (\x -> let i = 3 * (row * w + x)
                             in RGB (bytes SV.! i, bytes SV.! (i + 1), bytes SV.! (i + 2)))
  | row <- [0 .. h - 1] ]

-- | Drop-in for @runRender (mkRenderStaticEnv scene cam (w, h) ns maxDepth _) gens@
-- (src/Lib.hs:1491-1523): tier A, the reference's own stream layout — column x draws from gens !! x,
-- threaded down the column through every sample and bounce — so the bytes are the reference's
-- (within the transcendental-ulp tolerance of SURVEY.md §8d; DESIGN.md §4.5 gives the measured
-- agreement with a glibc-hosted reference). It is the EXACT mode, at CPU speed: a column is one serial
-- chain of draws, so only W lanes work (DESIGN.md §3.3); 'runRenderAMDPhilox' is the fast path. Like
-- runRender's VV.zip (src/Lib.hs:1519), a row holds min (length gens) w pixels: with fewer generators
-- than columns the rows are truncated (the missing columns are rendered with a copy of the first
-- generator and cut). One GPU (rt_create 0).
runRenderAMD :: Scene -> Camera -> (Int, Int) -> Int -> Int -> [RandGen] -> IO [VV.Vector RGB]
runRenderAMD scene cam (w, h) ns maxDepth gens = do
  let used = take w gens
      cols = Prelude.length used
  if cols == 0 || h <= 0
    then return (replicate (max 0 h) VV.empty)
    else do
      let padded = used ++ replicate (w - cols) (head used)
      bytes <- renderBytes 1 scene cam (w, h) ns maxDepth rtRngExact 0 (columnGens padded)
      return (toRows w h cols bytes)

-- | The fast path: tier B (one Philox4x32-10 stream per pixel and sample, keyed by `seed`), the
-- same image statistically (DESIGN.md §2, §4.6), full width, on one GPU.
runRenderAMDPhilox :: Scene -> Camera -> (Int, Int) -> Int -> Int -> Word64 -> IO [VV.Vector RGB]
runRenderAMDPhilox = runRenderAMDPhiloxOn 1

-- | 'runRenderAMDPhilox' over `gpus` GPUs of the node (opt-in): the image's tiles dealt round-robin
-- over the devices and gathered to the first with RCCL inside librtamd (rt_create_multi). The bytes
-- equal the one-GPU render's (tier B is shard-invariant). Its N > 1 path has run only where the GPU
-- box had one device (DESIGN.md §3.6).
runRenderAMDPhiloxOn :: Int -> Scene -> Camera -> (Int, Int) -> Int -> Int -> Word64 -> IO [VV.Vector RGB]
runRenderAMDPhiloxOn gpus scene cam (w, h) ns maxDepth seed = do
  bytes <- renderBytes gpus scene cam (w, h) ns maxDepth rtRngPhilox seed []
  return (toRows w h w bytes)
